# GPU: stacked-expert GEMM tests at Mixtral width, then full-width Mixtral-8x7B ZeRO-3 (8 of 32 layers) on 1 MI355X
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_moe_experts_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/moe_experts_gpu.log 2>&1 || exit 1
HDS_HANG_DUMP=60 timeout -k 10 420 python -u bench.py --model mixtral-8x7b --layers 8 --micro-batch 2 --steps 3 --warmup 1 > gpurun_out/mixtral_l8_mb2.log 2>&1 || exit 1
