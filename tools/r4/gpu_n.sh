# GPU: 320k ckpt_offload with a 225 GiB pinned-host budget (the default 160 GiB holds too few block inputs there)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4n
export HDS_BENCH_PROGRESS=1
timeout -k 10 900 python -u bench.py --seq 327680 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload --act-cache-host-gib 225 > gpurun_out/r4n/ckoff320k.log 2>&1
echo "rc=$?" >> gpurun_out/r4n/status.txt
