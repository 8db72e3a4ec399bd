# GPU: forward variant 11 with rolling per-fragment K ring in block A: parity, stamps, timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5aj
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and (10 or 11)" > $O/parity.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/fa_stamps.py 12 > $O/stamps.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,11,5,11,5,11 x > $O/fwd.log 2>&1 || exit 1
cat $O/stamps.log $O/fwd.log
