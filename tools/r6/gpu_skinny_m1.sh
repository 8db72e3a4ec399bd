# One-row decode linears (o, down, LM head at B = 1) on the skinny matrix-core GEMM vs the VALU GEMV / hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6skm1
mkdir -p $O
for t in 1 2 1 2; do
  HDS_SKINNY_MIN_M=$t timeout -k 10 300 python tools/bench_v2_decode.py --batches 1 --steps 128 > $O/decode_m${t}_$RANDOM.jsonl 2> $O/err_$t.log || { echo "decode failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/decode_m*.jsonl; do sed "s#^#$(basename $f) #" $f; done
