# GPU: MoE tests (per-expert GEMMs, in-place expert weight gradients) + Mixtral 8-layer mb4 throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_moe_experts_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/moe_experts_gpu2.log 2>&1 || exit 1
HDS_HANG_DUMP=60 timeout -k 10 420 python -u bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 3 --warmup 1 > gpurun_out/mixtral_l8_mb4_opt.log 2>&1 || exit 1
