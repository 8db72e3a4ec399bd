# GPU: FlashAttention built without SLP vectorization (no packed-f32 VALU beside the MFMAs) vs default: parity + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
AB=$GRAFT_REPO_ROOT/hcache_deepspeed_amd/_lib/ab/libhds_kernels.so
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
HDS_KERNEL_LIB=$AB timeout -k 10 300 $T tests/test_kernels_gpu.py -k "flash or attn" > gpurun_out/rp/flash_tests_ab.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rp/fa_bench_base.log 2>&1 || exit 1
HDS_KERNEL_LIB=$AB timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rp/fa_bench_ab.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rp/fa_bench_base2.log 2>&1 || exit 1
HDS_KERNEL_LIB=$AB timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rp/fa_bench_ab2.log 2>&1 || exit 1
HDS_KERNEL_LIB=$AB timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rp/bench_ab.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rp/bench_base.log 2>&1 || exit 1
