# GPU: budget-cap + transport-selection tests, then 512k tokens of Llama-3-8B (ckpt_offload + stash, default pinned
# budget; one warm-up + one timed step)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 500 python -u -m pytest tests/test_act_plan_gpu.py tests/test_transport_select_gpu.py tests/test_inference_v2.py -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
export HDS_BENCH_PROGRESS=1
run timeout -k 10 1000 python -u bench.py --seq 524288 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload > $O/ckoff512k.log 2>&1
free -g >> $O/status.txt
exit 0
