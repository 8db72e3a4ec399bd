set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_e2e_gpu.py tests/test_wmix_gemm.py tests/test_inference_v2_modules.py > gpurun_out/e2e_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/e2e_test.log; exit 1; }
timeout -k 10 300 python -u tools/bench_wmix.py > gpurun_out/wmix_bench.log 2>&1
