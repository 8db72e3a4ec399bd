# Longest context on one MI355X: Llama-3-8B at 640k tokens (655,360) with FPDT (64k segments, host-offloaded) and the
# host activation cache (ckpt_offload); one timed step, no warmup (a step is ~10 minutes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6l640
mkdir -p $O
HDS_BENCH_PROGRESS=1 timeout -k 10 1080 python bench.py --steps 1 --warmup 0 --seq 655360 --micro-batch 1 --fpdt-chunk 65536 --host-act-cache --act-cache-policy ckpt_offload > $O/l640k.json 2> $O/l640k.err || { echo failed; grep -v "^\[bench\]" $O/l640k.err | tail -20; exit 1; }
grep '^{' $O/l640k.json | cut -c1-900
