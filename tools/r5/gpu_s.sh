# GPU: one-slot software-pipelined exps (forward variant 11, dQ variant 1): parity + timing; then the mb10 allocator sweep
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "(staggered_variant and (10 or 11)) or dq_w64" > $O/parity.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,10,11,5,10,11 x > $O/fwd.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/bench_attn_bwd_dq.py 0,1,0,1 > $O/bwd.log 2>&1 || exit 1
cat $O/fwd.log $O/bwd.log
bash tools/r5/gpu_r.sh
