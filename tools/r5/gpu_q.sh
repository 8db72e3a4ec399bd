# GPU: one-wave-per-SIMD dQ kernel: parity (variants, fp32 reference), backward timing, counters
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dq_w64" > $O/parity.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_bwd_dq.py 0,1,0,1 > $O/bwd.log 2>&1 || exit 1
cat $O/bwd.log
