# GPU: one-wave dQ kernel with buffer-descriptor LDS-DMA; forward helper moved to the shared header
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ap
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dq_w64 or (staggered_variant and (11 or 20)) or flash_attn_varlen or padding_seq" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 300 python -u tools/bench_attn_bwd_dq.py 0,1,0,1,0,1 > $O/dq.log 2>&1 || exit 1
cat $O/dq.log
