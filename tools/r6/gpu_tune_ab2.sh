# headline bench with the full TunableOp table (tuning/, 22 signatures) vs the partial one of the first tuning run
# (profiles/r6/tunableop_partial_r6c.csv, 9 signatures; +0.5 % over no table), interleaved on one box.
# NOTE: profiles/ is in .gpurunignore, so the cp below failed on the box and the "partial" runs had no table at all
# (the library heuristic): the recorded A/B is full table vs none.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6tab2
mkdir -p $O /tmp/tp
cp profiles/r6/tunableop_partial_r6c.csv /tmp/tp/tunableop_results0.csv
for t in full partial full partial; do
  if [ $t = partial ]; then export PYTORCH_TUNABLEOP_FILENAME=/tmp/tp/tunableop_results%d.csv; else unset PYTORCH_TUNABLEOP_FILENAME; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_${t}_$RANDOM.json 2> $O/err_$t.log || { echo "bench $t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/bench_*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f', d['value'], d['extra']['tuned_gemm_table'])"; done
