set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kt2.log 2>&1 && \
timeout -k 10 300 python tools/bench_attn.py > gpurun_out/attn_bench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_full2.log 2>&1
echo "rc=$?" >> gpurun_out/bench_full2.log
