# v2 decode with HCache latent capture in the graph (hidden mode) vs capture off, B=1,4,8, on the round-6 kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6cap
mkdir -p $O
timeout -k 10 400 python tools/bench_v2_decode.py --capture-latents --batches 1,4,8 --steps 64 > $O/decode_capture.jsonl 2> $O/decode_capture.err || { echo failed; tail -20 $O/decode_capture.err; exit 1; }
cat $O/decode_capture.jsonl
