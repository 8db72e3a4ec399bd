# GPU: FlashAttention forward variant 8 (software-pipelined, 4-wave workgroups, two per CU) vs 5: parity + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rac
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "staggered_variant" > gpurun_out/rac/variant_tests.log 2>&1 || exit 1
for r in 1 2; do
  HDS_ATTN_FWD_VAR=5 timeout -k 10 200 python -u tools/r3/fa_bench.py --iters 10 > gpurun_out/rac/fa_v5_$r.log 2>&1 || exit 1
  HDS_ATTN_FWD_VAR=8 timeout -k 10 200 python -u tools/r3/fa_bench.py --iters 10 > gpurun_out/rac/fa_v8_$r.log 2>&1 || exit 1
done
