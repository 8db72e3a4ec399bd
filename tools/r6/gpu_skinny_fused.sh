# Decode steps of 2..16 tokens with the pre-norms / SwiGLU inside the skinny matrix-core GEMM: kernel + v2 GPU tests,
# then v2 decode B=1,4,8 with it (HDS_V2_FUSED_DECODE=1) and without (0), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6skf
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_v2.py -x -q --timeout 120 --timeout-method thread -k "skinny or gemv or hcache or decode or graph or latent" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 1 0 1 0; do
  HDS_V2_FUSED_DECODE=$t timeout -k 10 300 python tools/bench_v2_decode.py --batches 1,4,8 --steps 64 > $O/decode_f${t}_$RANDOM.jsonl 2> $O/err_$t.log || { echo "decode failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/decode_f*.jsonl; do sed "s#^#$(basename $f) #" $f; done
