# GPU: MX-FP8 LoRA test; bench with hipBLASLt forward GEMMs vs the hand-written MFMA forward GEMM (+ rocprof)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "lora_linear_mx or mx_" > gpurun_out/mxlin_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/mxlin_test.log; exit 1; }
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_lib.log 2>&1 || exit 1
HDS_GEMM_FWD=1 timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_gemmfwd.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_lib2.log 2>&1 || exit 1
HDS_GEMM_FWD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gf -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof_gf.log 2>&1 || exit 1
