# GPU: int8/int4 weight-only GEMV numerics + decode micro-benchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_int_gemv.py tests/test_inference_v1.py tests/test_kernels_gpu.py tests/test_fp_quantizer.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/intq_tests.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/intq_tests.log; exit 1; }
timeout -k 10 300 python -u tools/bench_int_gemv.py > gpurun_out/intq_bench.log 2>&1
