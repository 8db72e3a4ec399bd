# GPU: forward variant 12 cycle stamps; mb10 optimizer-state offload reloading during the one-rank backward
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5t
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 200 python -u tools/fa_stamps.py > $O/stamps.log 2>&1 || exit 1
cat $O/stamps.log
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.35 > $O/mb10_offstates_0.35.log 2>&1
export PYTORCH_HIP_ALLOC_CONF=expandable_segments:True
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.35 > $O/mb10_offstates_0.35_exp.log 2>&1
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.45 > $O/mb10_offstates_0.45_exp.log 2>&1
exit 0
