# Mixtral-8x7B (8 layers, mb4): the table with the Mixtral signatures (profiles/r6/tunableop_mixtral_r6e.csv) vs the
# committed Llama-only table (Mixtral GEMMs on the library heuristic), interleaved on one box
set -eo pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6tabmx2
mkdir -p $O /tmp/tmx
cp tools/r6/tunableop_mixtral_r6e.csv /tmp/tmx/tunableop_results0.csv  # profiles/ is not uploaded (the file now ships as tuning/)
for t in mx base mx base; do
  if [ $t = mx ]; then export PYTORCH_TUNABLEOP_FILENAME=/tmp/tmx/tunableop_results%d.csv; else unset PYTORCH_TUNABLEOP_FILENAME; fi
  timeout -k 10 300 python bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 6 --warmup 2 > $O/bench_${t}_$RANDOM.json 2> $O/err_$t.log || { echo "bench $t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/bench_*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f', d['value'])"; done
