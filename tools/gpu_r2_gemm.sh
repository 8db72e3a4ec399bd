# GPU: hand-written MFMA GEMM correctness + microbenchmark vs hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k 'gemm_nt or mx_' > gpurun_out/gemm_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/gemm_test.log; exit 1; }
timeout -k 10 300 python -u tools/bench_gemm.py 3 > gpurun_out/gemm_bench.log 2>&1 || { echo "rc=$?" >> gpurun_out/gemm_bench.log; exit 1; }
