# GPU: FA dK/dV with the pre-scaled LSE (delta pre-kernel writes lse*log2e): flash tests + timing + headline bench;
# host activation cache policy ckpt_offload: test, then Llama-3-8B at 32k / 128k / 256k tokens (micro-batch 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rs
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py tests/test_evoformer_gpu.py -k "flash or attn or evoformer" > gpurun_out/rs/flash_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rs/fa_bench.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rs/bench.log 2>&1 || exit 1
timeout -k 10 300 $T tests/test_host_tier_gpu.py > gpurun_out/rs/host_tier_tests.log 2>&1 || exit 1
export HDS_BENCH_PROGRESS=1
B="python -u bench.py --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload"
timeout -k 10 400 $B --seq 32768 --steps 3 --warmup 2 > gpurun_out/rs/ckoff_32k.log 2>&1 || exit 1
timeout -k 10 500 $B --seq 131072 --steps 2 --warmup 1 > gpurun_out/rs/ckoff_128k.log 2>&1 || exit 1
timeout -k 10 700 $B --seq 262144 --steps 1 --warmup 1 > gpurun_out/rs/ckoff_256k.log 2>&1 || exit 1
