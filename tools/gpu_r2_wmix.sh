set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_wmix_gemm.py tests/test_int_gemv.py tests/test_fp_quantizer.py tests/test_inference_v2_modules.py > gpurun_out/wmix_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/wmix_test.log; exit 1; }
timeout -k 10 300 python -u tools/bench_wmix.py > gpurun_out/wmix_bench.log 2>&1
