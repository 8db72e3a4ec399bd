set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --layers 4 --steps 3 --warmup 2 > gpurun_out/bench_l4.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_full.log 2>&1
echo "rc=$?" >> gpurun_out/bench_full.log
