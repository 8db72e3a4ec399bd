# Host activation cache controls (round 6, VERDICT r5 Next 7): plan vs recompute (fills the budget without spilling)
# at 32k x mb2 and 64k x mb1, default budget, one box. RUNS: "policy seq mb" triples separated by ';'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ctl
mkdir -p $O
IFS=';' read -ra LIST <<< "${RUNS:-plan 32768 2;recompute 32768 2;plan 65536 1;recompute 65536 1}"
for run in "${LIST[@]}"; do
  set -- $run
  f=$O/$1_$2_mb$3
  timeout -k 10 420 python bench.py --steps 4 --warmup 4 --seq $2 --micro-batch $3 --host-act-cache --act-cache-policy $1 > $f.json 2> $f.err || { echo "$run failed"; tail -20 $f.err; exit 1; }
  python tools/r6/ctl_summary.py $f.json "$run"
done
