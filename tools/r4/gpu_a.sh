# GPU: round-4 start: headline bench, FA micro-bench, 32k recompute baseline at 230 GiB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4a/bench.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/r3/fa_bench.py > gpurun_out/r4a/fa.log 2>&1 || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 4 --host-act-cache --act-cache-budget-gib 230"
timeout -k 10 500 $B --act-cache-policy recompute > gpurun_out/r4a/ac32k_b230_recompute.log 2>&1 || exit 1
