# GPU: 512k tokens of Llama-3-8B on one MI355X, ckpt_offload + attention stash, default pinned budget (first attempt:
# one warm-up and one timed step, to fit the call's time limit)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
export HDS_BENCH_PROGRESS=1
timeout -k 10 1140 python -u bench.py --seq 524288 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload > $O/ckoff512k.log 2>&1
echo "rc=$?" >> $O/status.txt
free -g >> $O/status.txt
