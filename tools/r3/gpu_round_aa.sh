# GPU: FlashAttention forward variant 7 (per-wave skip of causal tiles above its queries) vs 5: parity + timing + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/raa
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "staggered_variant" > gpurun_out/raa/variant_tests.log 2>&1 || exit 1
for r in 1 2; do
  HDS_ATTN_FWD_VAR=5 timeout -k 10 200 python -u tools/r3/fa_bench.py --iters 10 > gpurun_out/raa/fa_v5_$r.log 2>&1 || exit 1
  HDS_ATTN_FWD_VAR=7 timeout -k 10 200 python -u tools/r3/fa_bench.py --iters 10 > gpurun_out/raa/fa_v7_$r.log 2>&1 || exit 1
done
HDS_ATTN_FWD_VAR=7 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/raa/bench_v7.log 2>&1 || exit 1
HDS_ATTN_FWD_VAR=5 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/raa/bench_v5.log 2>&1 || exit 1
