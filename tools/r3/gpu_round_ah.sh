# GPU: 128k ckpt_offload with the activation-cache debug trace (prefetch issue / late-unpack times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rah
HDS_ACT_CACHE_DEBUG=1 HDS_BENCH_PROGRESS=1 timeout -k 10 500 python -u bench.py --seq 131072 --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload --steps 1 --warmup 1 > gpurun_out/rah/ckoff128k_debug.log 2>&1 || exit 1
