# GPU: 32k / 230 GiB with the one-step plan refinement (auto vs recompute), Mixtral-8x7B width (8 layers) re-measure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ry
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230"
timeout -k 10 500 $B --act-cache-policy auto > gpurun_out/ry/auto05.log 2>&1 || exit 1
timeout -k 10 500 $B --act-cache-policy recompute > gpurun_out/ry/recompute.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 4 --warmup 2 > gpurun_out/ry/mixtral_l8.log 2>&1 || exit 1
