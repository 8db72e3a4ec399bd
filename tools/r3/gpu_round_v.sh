# GPU: 32k host activation cache under a 230 GiB HBM budget with the round-3 end kernels: spill policy vs recompute
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rv
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 4 --host-act-cache --act-cache-budget-gib 230"
timeout -k 10 500 $B > gpurun_out/rv/ac32k_b230_spill.log 2>&1 || exit 1
timeout -k 10 500 $B --act-cache-policy recompute > gpurun_out/rv/ac32k_b230_recompute.log 2>&1 || exit 1
