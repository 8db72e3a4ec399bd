# GPU: long-context check of the final tree (forward variant 20 + buffer-descriptor DMA at 128k / 320k tokens)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ax
mkdir -p $O
export HDS_BENCH_PROGRESS=1
timeout -k 10 400 python -u bench.py --seq 131072 --micro-batch 1 --steps 3 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > $O/ckoff128k.log 2>&1
echo "128k rc=$?" >> $O/status.txt
grep -h metric $O/*.log
