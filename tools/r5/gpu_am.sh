# GPU: forward variant 11 with buffer-descriptor LDS-DMA (no per-tile offset clamps): parity, stamps, timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5an
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_attn or staggered_variant" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -3 $O/parity.log
timeout -k 10 200 python -u tools/fa_stamps.py 12 > $O/stamps.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,11,12,5,11,12,5,11 x > $O/fwd.log 2>&1 || exit 1
cat $O/stamps.log $O/fwd.log
