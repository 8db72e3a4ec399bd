# GPU: activation cache with a separate H2D prefetch stream: host-tier tests, 32k spill / auto at 230 GiB, 128k
# ckpt_offload with a kernel trace (compute gaps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rag
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_host_tier_gpu.py > gpurun_out/rag/host_tier_tests.log 2>&1 || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230"
timeout -k 10 500 $B > gpurun_out/rag/ac32k_b230_spill.log 2>&1 || exit 1
timeout -k 10 500 $B --act-cache-policy auto > gpurun_out/rag/ac32k_b230_auto.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rag/ckoff128k -o run -- python3 bench.py --seq 131072 --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload --steps 1 --warmup 1 > gpurun_out/rag/ckoff128k.log 2>&1 || exit 1
find gpurun_out/rag -name "*.csv" -size +20M -delete
