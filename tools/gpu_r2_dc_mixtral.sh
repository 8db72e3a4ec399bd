# GPU: DeepCompile ZeRO-Infinity schedule test, then Mixtral-8x7B full-width hang diagnosis at small depth
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_host_tier_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dc_gpu_test.log 2>&1 || exit 1
HDS_HANG_DUMP=60 timeout -k 10 240 python -u bench.py --model mixtral-8x7b --layers 2 --micro-batch 1 --steps 2 --warmup 1 > gpurun_out/mixtral_l2_mb1.log 2>&1 || exit 1
HDS_HANG_DUMP=60 timeout -k 10 300 python -u bench.py --model mixtral-8x7b --layers 8 --micro-batch 2 --steps 2 --warmup 1 > gpurun_out/mixtral_l8_mb2.log 2>&1 || exit 1
