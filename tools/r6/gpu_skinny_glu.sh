# SwiGLU in the skinny GEMM's epilogue for the gate|up projection at 2..16 decode rows: tests, then v2 decode B=4,8
# with (HDS_SKINNY_GLU=1) and without, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6skglu
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_v2.py -x -q --timeout 120 --timeout-method thread -k "skinny or gemv or hcache or decode or graph" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in 1 0 1 0; do
  HDS_SKINNY_GLU=$t timeout -k 10 300 python tools/bench_v2_decode.py --batches 4,8 --steps 64 > $O/decode_g${t}_$RANDOM.jsonl 2> $O/err_$t.log || { echo "decode failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/decode_g*.jsonl; do sed "s#^#$(basename $f) #" $f; done
