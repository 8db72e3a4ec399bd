# v2 decode with HCache latent capture in the graph (hidden mode) vs capture off, B=1,4,8, on the round-6 kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6cap${TAG:-}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_inference_v2.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "hcache or decode or graph or latent or gemv" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python tools/bench_v2_decode.py --capture-latents --batches 1,4,8 --steps 64 > $O/decode_capture.jsonl 2> $O/decode_capture.err || { echo failed; tail -20 $O/decode_capture.err; exit 1; }
cat $O/decode_capture.jsonl
