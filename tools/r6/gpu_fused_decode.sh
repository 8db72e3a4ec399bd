# Decode GEMVs with the RMSNorm / SwiGLU folded in: kernel + v2 GPU tests, then v2 decode B=1,4,8 fused vs unfused
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6fdec
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_v2.py -x -v --timeout 120 --timeout-method thread -k "gemv or hcache or decode or latent or graph" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in 1 0; do
  HDS_V2_FUSED_DECODE=$t timeout -k 10 300 python tools/bench_v2_decode.py --batches 1,4,8 --steps 64 > $O/decode_fused$t.jsonl 2> $O/decode_fused$t.err || { echo "decode $t failed"; tail -20 $O/decode_fused$t.err; exit 1; }
  sed "s/^/fused=$t /" $O/decode_fused$t.jsonl
done
