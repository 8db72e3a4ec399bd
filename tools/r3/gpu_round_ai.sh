# GPU: activation cache -- kept blocks tagged, own-block prefetch first: host-tier tests, 128k ckpt_offload kernel trace
# (compute gaps), 32k / 230 GiB spill and auto
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rai
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_host_tier_gpu.py > gpurun_out/rai/host_tier_tests.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rai/ckoff128k -o run -- python3 bench.py --seq 131072 --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload --steps 1 --warmup 1 > gpurun_out/rai/ckoff128k.log 2>&1 || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230"
timeout -k 10 500 $B > gpurun_out/rai/ac32k_b230_spill.log 2>&1 || exit 1
timeout -k 10 500 $B --act-cache-policy auto > gpurun_out/rai/ac32k_b230_auto.log 2>&1 || exit 1
find gpurun_out/rai -name "*.csv" -size +20M -delete
