# GPU: final full GPU test suite + smoke on the round-3 end tree, then FA forward variant 7 vs 5 (timing + bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/rab/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/rab/smoke.log 2>&1 || exit 1
for r in 1 2; do
  HDS_ATTN_FWD_VAR=5 timeout -k 10 200 python -u tools/r3/fa_bench.py --iters 10 > gpurun_out/rab/fa_v5_$r.log 2>&1 || exit 1
  HDS_ATTN_FWD_VAR=7 timeout -k 10 200 python -u tools/r3/fa_bench.py --iters 10 > gpurun_out/rab/fa_v7_$r.log 2>&1 || exit 1
done
HDS_ATTN_FWD_VAR=7 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rab/bench_v7.log 2>&1 || exit 1
HDS_ATTN_FWD_VAR=5 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rab/bench_v5.log 2>&1 || exit 1
