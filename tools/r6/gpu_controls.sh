# Host activation cache controls (round 6, VERDICT r5 Next 7): plan vs recompute (fills the budget without spilling)
# at 32k x mb2 and 64k x mb1, default budget, one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ctl
mkdir -p $O
for cfg in "32768 2" "65536 1"; do
  set -- $cfg
  for pol in plan recompute; do
    timeout -k 10 420 python bench.py --steps 4 --warmup 3 --seq $1 --micro-batch $2 --host-act-cache --act-cache-policy $pol > $O/${pol}_$1_mb$2.json 2> $O/${pol}_$1_mb$2.err || { echo "$pol $1 failed"; tail -20 $O/${pol}_$1_mb$2.err; exit 1; }
    python -c "import json;d=json.loads([l for l in open('$O/${pol}_$1_mb$2.json') if l.startswith('{')][-1]);a=d['extra'].get('act_cache',{});print('$pol $1 mb$2', d['value'], d['extra'].get('peak_gib_timed_steps'), a.get('bytes_offloaded'), a.get('recomputed_layers'))"
  done
done
