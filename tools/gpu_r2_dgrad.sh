set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_wgrad_layout_gpu.py tests/test_kernels_gpu.py tests/test_e2e_gpu.py > gpurun_out/wgrad_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/wgrad_test.log; exit 1; }
timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_dgrad_auto.log 2>&1 || exit 1
HDS_DGRAD_LAYOUT=direct timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_dgrad_direct.log 2>&1 || exit 1
