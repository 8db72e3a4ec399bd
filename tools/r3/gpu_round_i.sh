# GPU: 32k host activation cache at a 230 GiB budget -- prefetch headroom, expandable allocator segments A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ri
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 3"
timeout -k 10 500 $B --host-act-cache --act-cache-budget-gib 230 > gpurun_out/ri/ac32k_b230.log 2>&1 || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 500 $B --host-act-cache --act-cache-budget-gib 230 > gpurun_out/ri/ac32k_b230_exp.log 2>&1 || exit 1
timeout -k 10 500 $B --ckpt > gpurun_out/ri/ckpt32k.log 2>&1 || exit 1
