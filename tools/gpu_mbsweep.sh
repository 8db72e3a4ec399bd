# GPU: micro-batch sweep of the headline bench (memory headroom on 288 GB)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --micro-batch 7 > gpurun_out/bench_mb7.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --micro-batch 8 > gpurun_out/bench_mb8.log 2>&1
