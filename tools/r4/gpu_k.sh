# GPU: when does the HIP runtime read DEBUG_CLR_LIMIT_BLIT_WG (probe); 32k plan through bench.py (which now sets it
# before importing torch) plus a kernel-only trace of it; optimizer-state offload of one state (ratio 0.3) at mb10
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4k/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run timeout -k 10 120 python -u tools/r4/blit_env_probe.py none > gpurun_out/r4k/probe.log 2>&1
run timeout -k 10 120 python -u tools/r4/blit_env_probe.py late >> gpurun_out/r4k/probe.log 2>&1
DEBUG_CLR_LIMIT_BLIT_WG=16 run timeout -k 10 120 python -u tools/r4/blit_env_probe.py >> gpurun_out/r4k/probe.log 2>&1
export HDS_BENCH_PROGRESS=1
P="python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8"
run timeout -k 10 300 $P --steps 4 --warmup 5 > gpurun_out/r4k/plan32k.log 2>&1
export DEBUG_CLR_LIMIT_BLIT_WG=16
run timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4k/plan32k -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8 --steps 1 --warmup 5 > gpurun_out/r4k/plan32k_trace.log 2>&1
unset DEBUG_CLR_LIMIT_BLIT_WG
run python3 tools/r4/step_timeline.py gpurun_out/r4k/plan32k > gpurun_out/r4k/plan32k_timeline.txt 2>&1
run python3 tools/r3/trace_step_stats.py gpurun_out/r4k/plan32k > gpurun_out/r4k/plan32k_kernels.txt 2>&1
find gpurun_out/r4k -name "*.csv" -size +40M -delete
run timeout -k 10 300 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states --offload-states-ratio 0.3 > gpurun_out/r4k/mb10_offstates030.log 2>&1
run timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4k/head -o run -- python3 bench.py --steps 3 --warmup 3 > gpurun_out/r4k/head_trace.log 2>&1
run python3 tools/r3/trace_step_stats.py gpurun_out/r4k/head > gpurun_out/r4k/head_kernels.txt 2>&1
find gpurun_out/r4k -name "*.csv" -size +40M -delete
