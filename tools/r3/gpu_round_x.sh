# GPU: 32k under a 230 GiB HBM budget -- host activation cache policy auto (recompute, then the earliest blocks spill
# as far as PCIe hides them) at two overlap fractions vs recompute, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rx
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_host_tier_gpu.py > gpurun_out/rx/host_tier_tests.log 2>&1 || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230"
timeout -k 10 500 $B --act-cache-policy auto > gpurun_out/rx/auto05.log 2>&1 || exit 1
timeout -k 10 500 $B --act-cache-policy auto --act-cache-spill-overlap 0.3 > gpurun_out/rx/auto03.log 2>&1 || exit 1
timeout -k 10 500 $B --act-cache-policy recompute > gpurun_out/rx/recompute.log 2>&1 || exit 1
