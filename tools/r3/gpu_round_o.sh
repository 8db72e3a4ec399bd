# GPU: producer-written transposes (glu fwd/bwd), batched split-K wgrad default, GLU v2 kernels; tests, micro-benchmarks,
# headline bench + kernel profile of the step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ro
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_wgrad_layout_gpu.py > gpurun_out/ro/wgrad_tests.log 2>&1 || exit 1
timeout -k 10 300 $T tests/test_kernels_gpu.py -k glu > gpurun_out/ro/glu_tests.log 2>&1 || exit 1
timeout -k 10 400 $T tests/test_grad_parity_gpu.py tests/test_e2e_gpu.py > gpurun_out/ro/parity_tests.log 2>&1 || exit 1
HDS_GLU_VAR=1 timeout -k 10 120 python -u tools/bench_glu.py > gpurun_out/ro/glu_bench.log 2>&1 || exit 1
HDS_GLU_VAR=2 timeout -k 10 120 python -u tools/bench_glu.py >> gpurun_out/ro/glu_bench.log 2>&1 || exit 1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/ro/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ro/bench.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ro/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/ro/prof_bench.log 2>&1 || exit 1
python tools/r3/glue_census.py gpurun_out/ro/prof > gpurun_out/ro/glue_census.txt 2>&1
python tools/r3/trace_step_stats.py gpurun_out/ro/prof > gpurun_out/ro/step_stats.txt 2>&1
find gpurun_out/ro/prof -name "*kernel_trace.csv" -size +20M -delete
