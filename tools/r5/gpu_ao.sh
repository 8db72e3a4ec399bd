# GPU: forward variants 18 (DMA spread over block A) and 20 (+ first V group read in block A): parity, stamps, timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ao
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and (11 or 18 or 20)" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 200 python -u tools/fa_stamps.py 12 > $O/stamps.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/fa_stamps.py 19 >> $O/stamps.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/fa_stamps.py 21 >> $O/stamps.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 11,18,20,11,18,20,11,18,20 x > $O/fwd.log 2>&1 || exit 1
cat $O/stamps.log $O/fwd.log
