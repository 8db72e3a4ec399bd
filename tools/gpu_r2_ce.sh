# GPU: LM-head + CE chunk size A/B inside the full training step (first-chunk beta=0 in all runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "cross_entropy or xent or fused" > gpurun_out/ce_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/ce_test.log; exit 1; }
for c in 4096 8192 14336; do
  HDS_CE_CHUNK_ROWS=$c timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_ce_$c.log 2>&1 || exit 1
done
