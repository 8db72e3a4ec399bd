set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HDS_BENCH_PROGRESS=1 HDS_ACT_CACHE_DEBUG=1
mkdir -p gpurun_out/actc
timeout -k 10 400 python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --steps 2 --warmup 2 > gpurun_out/actc/bench4.log 2>&1 || exit 1
