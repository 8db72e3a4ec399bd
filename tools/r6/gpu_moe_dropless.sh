# Mixtral-8x7B (8 layers, mb4): dropless (capacity = the step's largest expert load, GEMMs over occupied slots) vs
# capacity factor 1.25 with token dropping, interleaved on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6moedl
mkdir -p $O
for t in dl cap dl cap; do
  X=""; [ $t = dl ] && X="--moe-dropless"
  timeout -k 10 300 python bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 6 --warmup 3 $X > $O/bench_${t}_$RANDOM.json 2> $O/err_$t.log || { echo "bench $t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/bench_*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f', d['value'], d['extra'].get('peak_mem_gib'), d['extra'].get('final_loss'))"; done
