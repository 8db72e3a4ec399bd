# Headline with / without the batched two-half weight-gradient candidates (HDS_WGRAD_B2) in the layout tuner,
# interleaved on one box; the chosen layouts are printed per run (HDS_GEMM_LAYOUT_LOG=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6b2
mkdir -p $O
for t in 1 0 1 0; do
  HDS_WGRAD_B2=$t timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_b2${t}_$RANDOM.json 2> $O/err_$t.log || { echo "bench $t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/bench_b2*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f', d['value'])"; done
