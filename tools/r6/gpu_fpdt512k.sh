# FPDT attention in the Llama-3-8B model at 512k tokens on one MI355X (round 6, VERDICT r5 Next 2), with the host
# activation cache (ckpt_offload); compare with ckpt_offload alone (profiles/r5/ckoff512k_r5d.json: 1,438 tok/s)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6fpdt
mkdir -p $O
HDS_BENCH_PROGRESS=1 timeout -k 10 1100 python bench.py --steps 1 --warmup 1 --seq 524288 --micro-batch 1 --fpdt-chunk ${CHUNK:-65536} ${FPDT_EXTRA:-} --host-act-cache --act-cache-policy ckpt_offload > $O/fpdt512k${TAG:-}.json 2> $O/fpdt512k${TAG:-}.err || { echo failed; tail -30 $O/fpdt512k${TAG:-}.err; exit 1; }
cat $O/fpdt512k${TAG:-}.json
