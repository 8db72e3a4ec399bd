# headline bench with / without the committed TunableOp table (tuning/tunableop_results0.csv), interleaved on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6tab
mkdir -p $O
for t in 1 0 1 0; do
  HDS_TUNABLEOP=$t timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_tuned${t}_$RANDOM.json 2> $O/err_$t.log || { echo "bench $t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/bench_tuned*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f', d['value'], d['extra']['tuned_gemm_table'])"; done
