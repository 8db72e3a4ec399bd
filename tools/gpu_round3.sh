# GPU: full gpu test suite, default bench (mb6) and a rocprofv3 kernel-stats profile of it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests3.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/gpu_tests3.log; exit 1; }
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_r3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3 -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_r3.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof_r3.log
