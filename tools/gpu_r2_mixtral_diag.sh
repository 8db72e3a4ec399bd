# GPU: locate the Mixtral full-width stall: every native launch synchronised, stacks dumped every 20 s
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HDS_DEBUG_SYNC=1 AMD_SERIALIZE_KERNEL=3 HDS_HANG_DUMP=20 timeout -k 10 100 python -u bench.py --model mixtral-8x7b --layers 1 --micro-batch 1 --seq 1024 --steps 1 --warmup 1 > gpurun_out/mixtral_diag_s1024.log 2>&1 || exit 1
HDS_DEBUG_SYNC=1 AMD_SERIALIZE_KERNEL=3 HDS_HANG_DUMP=20 timeout -k 10 100 python -u bench.py --model mixtral-8x7b --layers 1 --micro-batch 1 --steps 1 --warmup 1 > gpurun_out/mixtral_diag.log 2>&1 || exit 1
