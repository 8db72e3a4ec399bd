# GPU: 32k plan with only the package's blit default (no env) + a trace with the limit exported for the profiler
# (rocprofv3 initialises HIP before the package is imported); optimizer-state offload at ratios 0.5 (two of the three states) / 0.34 (one) at mb10;
# HCache int8 latents (test + restore bench)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4h/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
export HDS_BENCH_PROGRESS=1
P="python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8"
run timeout -k 10 300 $P --steps 4 --warmup 5 > gpurun_out/r4h/plan32k_pkgdefault.log 2>&1
export DEBUG_CLR_LIMIT_BLIT_WG=16
run timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4h/plan32k -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8 --steps 1 --warmup 5 > gpurun_out/r4h/plan32k_trace.log 2>&1
unset DEBUG_CLR_LIMIT_BLIT_WG
run python3 tools/r4/step_timeline.py gpurun_out/r4h/plan32k > gpurun_out/r4h/plan32k_timeline.txt 2>&1
run python3 tools/r3/trace_step_stats.py gpurun_out/r4h/plan32k > gpurun_out/r4h/plan32k_kernels.txt 2>&1
find gpurun_out/r4h -name "*.csv" -size +40M -delete
run timeout -k 10 300 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states --offload-states-ratio 0.5 > gpurun_out/r4h/mb10_offstates050.log 2>&1
run timeout -k 10 300 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states --offload-states-ratio 0.34 > gpurun_out/r4h/mb10_offstates034.log 2>&1
run timeout -k 10 200 python -u -m pytest tests/test_inference_v2.py -k quantized_latents -x -v --timeout 120 --timeout-method thread > gpurun_out/r4h/v2_latent_tests.log 2>&1
run timeout -k 10 400 python -u tools/bench_hcache.py --seqs 8 --ctx 2048 > gpurun_out/r4h/hcache.log 2>&1
