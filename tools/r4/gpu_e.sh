# GPU: few-workgroup D2H copy kernel for activation spills -- tests, then 32k plan with it (16 / 8 workgroups) and with
# the runtime blit limited by DEBUG_CLR_LIMIT_BLIT_WG; optimizer-state offload at mb10 (states off the device from the start)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4e/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run timeout -k 10 300 python -u -m pytest tests/test_host_tier_gpu.py tests/test_act_plan_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4e/tests.log 2>&1
grep -q "failed" gpurun_out/r4e/tests.log && exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230 --act-cache-policy plan --act-cache-spill-overlap 0.8"
run timeout -k 10 300 $B > gpurun_out/r4e/plan_wg16.log 2>&1
HDS_D2H_WG=8 run timeout -k 10 300 $B > gpurun_out/r4e/plan_wg8.log 2>&1
HDS_D2H_WG=0 DEBUG_CLR_LIMIT_BLIT_WG=16 run timeout -k 10 300 $B > gpurun_out/r4e/plan_blit16.log 2>&1
run timeout -k 10 300 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states > gpurun_out/r4e/mb10_offstates100.log 2>&1
