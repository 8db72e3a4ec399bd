# GPU: 32k Llama-3-8B host activation cache regression diagnosis (allocator retries, late unpacks, guard spills)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --steps 3 --warmup 2"
timeout -k 10 400 $B > gpurun_out/r3_32k_ac.log 2>&1 || exit 1
HDS_ACT_CACHE_DEBUG=1 timeout -k 10 400 $B --act-cache-budget-gib 230 > gpurun_out/r3_32k_ac230.log 2> gpurun_out/r3_32k_ac230.err || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 400 $B --act-cache-budget-gib 230 > gpurun_out/r3_32k_ac230_exp.log 2>&1 || exit 1
HDS_WGRAD_LAYOUT=direct HDS_DGRAD_LAYOUT=direct timeout -k 10 400 $B --act-cache-budget-gib 230 > gpurun_out/r3_32k_ac230_direct.log 2>&1 || exit 1
