# GPU: 256k ckpt_offload with the attention stash under the default pinned-host budget
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4y
export HDS_BENCH_PROGRESS=1
timeout -k 10 700 python -u bench.py --seq 262144 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload > gpurun_out/r4y/ckoff256k.log 2>&1
echo "rc=$?" >> gpurun_out/r4y/status.txt
