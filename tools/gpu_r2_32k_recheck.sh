# GPU: 32k-context Llama-3-8B, host activation cache vs activation checkpointing, on the session-end tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --steps 3 --warmup 2 > gpurun_out/r2_end_32k_actcache.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --seq 32768 --micro-batch 1 --ckpt --steps 3 --warmup 2 > gpurun_out/r2_end_32k_ckpt.log 2>&1 || exit 1
