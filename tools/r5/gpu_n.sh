# GPU: mb10 byte-granular optimizer-state offload with chunked tails (1 GiB), paced forward
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
for r in 0.35 0.45; do
  run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio $r > $O/mb10_offstates_$r.log 2>&1
done
exit 0
