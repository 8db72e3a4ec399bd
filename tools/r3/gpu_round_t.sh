# GPU: long context on one MI355X -- checkpointing alone at 128k (current kernels) vs ckpt_offload, and ckpt_offload
# at 320k tokens (pinned host use ~160 GB, inside the default host budget)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export HDS_BENCH_PROGRESS=1
mkdir -p gpurun_out/rt
timeout -k 10 500 python -u bench.py --micro-batch 1 --ckpt --seq 131072 --steps 1 --warmup 1 > gpurun_out/rt/ckpt_128k.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload --seq 327680 --steps 1 --warmup 1 > gpurun_out/rt/ckoff_320k.log 2>&1 || exit 1
