# GPU: FA forward variant 5 (pipelined softmax, immediate LDS offsets, DMA fast path) parity + timing, then round D
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rf
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "staggered_variant" > gpurun_out/rf/fa_var_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_attn_fwd_variants.py > gpurun_out/rf/fa_var_bench.log 2>&1 || exit 1
bash tools/r3/gpu_round_d.sh
