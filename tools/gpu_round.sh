# GPU round: all gpu tests, then bench variants
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 600 python bench.py --steps 6 --warmup 3 --micro-batch 4 > gpurun_out/bench_mb4.log 2>&1
echo "rc=$?" >> gpurun_out/bench_mb4.log
