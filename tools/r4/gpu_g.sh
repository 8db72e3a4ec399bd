# GPU: 128k long context -- ckpt_offload with the attention stash vs without vs plain checkpointing; 32k plan trace with
# the blit limit; GPU tests of the cache
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# the package sets DEBUG_CLR_LIMIT_BLIT_WG=16 itself
mkdir -p gpurun_out/r4g
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4g/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run timeout -k 10 300 python -u -m pytest tests/test_host_tier_gpu.py tests/test_act_plan_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4g/tests.log 2>&1
export HDS_BENCH_PROGRESS=1
L="python -u bench.py --seq 131072 --micro-batch 1 --steps 2 --warmup 2"
run timeout -k 10 400 $L --host-act-cache --act-cache-policy ckpt_offload > gpurun_out/r4g/ckoff128k_stash.log 2>&1
run timeout -k 10 400 $L --ckpt > gpurun_out/r4g/ckpt128k.log 2>&1
run timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4g/plan32k -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8 --steps 1 --warmup 5 > gpurun_out/r4g/plan32k_trace.log 2>&1
run python3 tools/r4/step_timeline.py gpurun_out/r4g/plan32k > gpurun_out/r4g/plan32k_timeline.txt 2>&1
run python3 tools/r3/trace_step_stats.py gpurun_out/r4g/plan32k > gpurun_out/r4g/plan32k_kernels.txt 2>&1
find gpurun_out/r4g -name "*.csv" -size +40M -delete
run timeout -k 10 300 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states > gpurun_out/r4g/mb10_offstates100.log 2>&1
