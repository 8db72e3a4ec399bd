# GPU: full-width Mixtral-8x7B (8 of 32 layers) ZeRO-3 on 1 MI355X: micro-batch 4 throughput + rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_mx
HDS_HANG_DUMP=60 timeout -k 10 420 python -u bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 3 --warmup 1 > gpurun_out/mixtral_l8_mb4.log 2>&1 || exit 1
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mx -o mx -- python3 bench.py --model mixtral-8x7b --layers 8 --micro-batch 2 --steps 2 --warmup 1 > gpurun_out/prof_mx.log 2>&1 || exit 1
find gpurun_out/prof_mx -name "*kernel_trace.csv" -size +20M -delete
