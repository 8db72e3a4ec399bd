# GPU: forward variant 10 after spreading the LDS-DMA pieces over block B: parity + TF/s vs 5
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and (10 or 11)" > $O/parity.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,10,11,5,10,11,5,11 x > $O/tfs.log 2>&1 || exit 1
cat $O/tfs.log
