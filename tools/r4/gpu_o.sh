# GPU: 320k ckpt_offload without the attention stash, then with it under expandable segments
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4o
export HDS_BENCH_PROGRESS=1
timeout -k 10 600 python -u bench.py --seq 327680 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload --act-cache-host-gib 225 --no-attn-stash > gpurun_out/r4o/ckoff320k_nostash.log 2>&1
rc=$?; echo "nostash rc=$rc" >> gpurun_out/r4o/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
PYTORCH_ALLOC_CONF=expandable_segments:True timeout -k 10 500 python -u bench.py --seq 327680 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload --act-cache-host-gib 225 > gpurun_out/r4o/ckoff320k_stash_expseg.log 2>&1
echo "stash_expseg rc=$?" >> gpurun_out/r4o/status.txt
