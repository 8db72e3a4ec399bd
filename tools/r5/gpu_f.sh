# GPU: HCache-on decode at graph speed (tools/bench_v2_decode.py --capture-latents); mb10 optimizer-state offload,
# byte-granular, against ZeRO-Offload CPU Adam on the same box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 400 python -u tools/bench_v2_decode.py --capture-latents > $O/decode_capture.jsonl 2> $O/decode_capture.err
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run timeout -k 10 300 $B --offload cpu > $O/mb10_zero_offload.log 2>&1
for r in 0.2 0.25; do
  run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio $r > $O/mb10_offstates_$r.log 2>&1
done
export HDS_BENCH_PROGRESS=1
run timeout -k 10 420 python -u bench.py --seq 65536 --micro-batch 1 --steps 4 --warmup 6 --host-act-cache --act-cache-policy plan --act-cache-spill-overlap 0.8 > $O/plan_65536_mb1.log 2>&1
exit 0
