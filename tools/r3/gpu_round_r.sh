# GPU: host activation cache policy ckpt_offload (every block checkpointed, inputs spilled to pinned host):
# test, then Llama-3-8B at 32k / 128k / 256k tokens (micro-batch 1) -- max sequence length at fixed HBM
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export HDS_BENCH_PROGRESS=1
mkdir -p gpurun_out/rr
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_host_tier_gpu.py > gpurun_out/rr/host_tier_tests.log 2>&1 || exit 1
B="python -u bench.py --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload"
timeout -k 10 400 $B --seq 32768 --steps 3 --warmup 2 > gpurun_out/rr/ckoff_32k.log 2>&1 || exit 1
timeout -k 10 500 $B --seq 131072 --steps 2 --warmup 1 > gpurun_out/rr/ckoff_128k.log 2>&1 || exit 1
timeout -k 10 700 $B --seq 262144 --steps 1 --warmup 1 > gpurun_out/rr/ckoff_256k.log 2>&1 || exit 1
