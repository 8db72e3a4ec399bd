# GPU: FlashAttention backward PIPE 2 (uniform-base LDS-DMA of full Q/dO and K/V tiles) vs PIPE 1, both built without
# SLP vectorization: parity (flash tests under PIPE 2) + timing + headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rq
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
HDS_ATTN_BWD_PIPE=2 timeout -k 10 300 $T tests/test_kernels_gpu.py -k "flash or attn" > gpurun_out/rq/flash_tests_pipe2.log 2>&1 || exit 1
HDS_ATTN_BWD_PIPE=1 timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rq/fa_bench_pipe1.log 2>&1 || exit 1
HDS_ATTN_BWD_PIPE=2 timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rq/fa_bench_pipe2.log 2>&1 || exit 1
HDS_ATTN_BWD_PIPE=1 timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rq/fa_bench_pipe1b.log 2>&1 || exit 1
HDS_ATTN_BWD_PIPE=2 timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rq/fa_bench_pipe2b.log 2>&1 || exit 1
HDS_ATTN_BWD_PIPE=2 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rq/bench_pipe2.log 2>&1 || exit 1
HDS_ATTN_BWD_PIPE=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rq/bench_pipe1.log 2>&1 || exit 1
