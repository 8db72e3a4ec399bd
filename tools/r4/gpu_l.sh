# GPU: 32k plan with the capacity back-off (closed loop) -- two bench runs + a kernel-only trace; act-plan GPU tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4l
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4l/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run timeout -k 10 300 python -u -m pytest tests/test_act_plan_gpu.py tests/test_host_tier_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4l/tests.log 2>&1
export HDS_BENCH_PROGRESS=1
P="python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8"
run timeout -k 10 300 $P --steps 6 --warmup 6 > gpurun_out/r4l/plan32k_a.log 2>&1
run timeout -k 10 300 python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy recompute --act-cache-budget-gib 230 --steps 4 --warmup 3 > gpurun_out/r4l/recompute32k.log 2>&1
run timeout -k 10 300 $P --steps 6 --warmup 6 > gpurun_out/r4l/plan32k_b.log 2>&1
export DEBUG_CLR_LIMIT_BLIT_WG=16
run timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4l/plan32k -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8 --steps 1 --warmup 8 > gpurun_out/r4l/plan32k_trace.log 2>&1
unset DEBUG_CLR_LIMIT_BLIT_WG
run python3 tools/r4/step_timeline.py gpurun_out/r4l/plan32k > gpurun_out/r4l/plan32k_timeline.txt 2>&1
find gpurun_out/r4l -name "*.csv" -size +40M -delete
