# Decode combine kernel with LDS-staged split stats: paged decode GPU tests, then v2 decode B=1,4,8 (compare with
# profiles/r6/decode_merge/decode_merge0_*.jsonl, the previous combine on the same code otherwise)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6comb
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_v2.py -x -v --timeout 120 --timeout-method thread -k "paged or hcache or decode or graph" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python tools/bench_v2_decode.py --batches 1,4,8 --steps 64 > $O/decode_$i.jsonl 2> $O/decode_$i.err || { echo "decode failed"; tail -20 $O/decode_$i.err; exit 1; }
  cat $O/decode_$i.jsonl
done
