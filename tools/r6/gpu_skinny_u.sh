# Skinny GEMM with 16 vs 8 weight loads per lane in flight (HDS_SKINNY_U), v2 decode B=4,8 interleaved, after its test
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6sku${TAG:-}
mkdir -p $O
HDS_SKINNY_U=${TU:-16} timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "skinny" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in ${US:-16 8 16 8}; do
  HDS_SKINNY_U=$t timeout -k 10 300 python tools/bench_v2_decode.py --batches 4,8 --steps 64 > $O/decode_u${t}_$RANDOM.jsonl 2> $O/err_$t.log || { echo "decode failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/decode_u*.jsonl; do sed "s#^#$(basename $f) #" $f; done
