# The plan policy at 32k x mb2 on the round-5 tree (_r5tree, a git worktree of 19eedca with its own built libraries)
# and on this tree, interleaved on one box: is the round-6 drop (13,093-13,442 -> 12,862-12,884 tok/s) code or box?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6r5
mkdir -p $O
for t in r5 head r5 head; do
  if [ $t = r5 ]; then D=$GRAFT_REPO_ROOT/_r5tree; else D=$GRAFT_REPO_ROOT; fi
  (cd $D && HDS_TUNABLEOP=0 timeout -k 10 300 python bench.py --steps 4 --warmup 4 --seq 32768 --micro-batch 2 --host-act-cache --act-cache-policy plan > $O/plan_${t}_$RANDOM.json 2> $O/err_$t.log) || { echo "$t failed"; tail -20 $O/err_$t.log; exit 1; }
done
for f in $O/plan_*.json; do python -c "import json;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);a=d['extra'].get('act_cache',{});print('$f', d['value'], a.get('throttle_wait_s'), a.get('t_fwd_ms'), a.get('spill_cost_measured'))"; done
