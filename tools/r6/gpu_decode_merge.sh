# Split-K paged decode with the split merge in the same launch (last workgroup merges): kernel + v2 GPU tests, then
# v2 decode B=1,4,8 with the in-kernel merge vs the separate combine launch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6merge
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_inference_v2.py -x -v --timeout 120 --timeout-method thread -k "paged or gemv or hcache or decode or latent or graph" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in 1 0 1; do  # 1: in-kernel merge (opt-in)
  HDS_DECODE_MERGE_IN_KERNEL=$t timeout -k 10 300 python tools/bench_v2_decode.py --batches 1,4,8 --steps 64 > $O/decode_merge${t}_$RANDOM.jsonl 2> $O/decode_merge$t.err || { echo "decode $t failed"; tail -20 $O/decode_merge$t.err; exit 1; }
done
for f in $O/decode_merge*.jsonl; do sed "s#^#$(basename $f) #" $f; done
