# GPU: SwiGLU kernel micro-bench + activation kernel tests + short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_glu.py > gpurun_out/glu_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_kernels_glu.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_glu.log 2>&1
