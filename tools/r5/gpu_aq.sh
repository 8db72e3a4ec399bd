# GPU: forward variant 22 (20 + s_setprio by wave index)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5aq
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and (20 or 22)" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 200 python -u tools/fa_stamps.py 21 > $O/stamps.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/fa_stamps.py 23 >> $O/stamps.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 20,22,20,22,20,22 x > $O/fwd.log 2>&1 || exit 1
cat $O/stamps.log $O/fwd.log
