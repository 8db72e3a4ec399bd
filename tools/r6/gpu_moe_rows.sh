# Mixtral-8x7B (8 layers, mb4): expert GEMMs over the occupied capacity slots only (HDS_MOE_EXACT_ROWS=1, default)
# vs every slot, interleaved on one box, after the MoE GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6moe${TAG:-}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_moe_experts_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in 1 0 1 0; do
  HDS_MOE_EXACT_ROWS=$t timeout -k 10 300 python bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 6 --warmup 3 > $O/bench_rows${t}_$RANDOM.json 2> $O/err_$t.log || { echo "bench $t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/bench_rows*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$f', d['value'], d['extra'].get('final_loss'))"; done
