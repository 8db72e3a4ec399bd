# GPU: budget-cap test (plan / recompute, feasible budget); plan at 32k x mb2 and 64k x mb1 (default budget) after the
# backward-excess fix; control: ckpt_offload with a ~0 pinned budget (checkpointing + attention stash kept on the
# device, nothing spilled) to separate the stash's gain from the spill's
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 300 python -u -m pytest tests/test_act_plan_gpu.py -k budget_is_a_cap -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1
export HDS_BENCH_PROGRESS=1
for shape in "32768 2" "65536 1"; do
  set -- $shape
  S=$1; MB=$2
  run timeout -k 10 420 python -u bench.py --seq $S --micro-batch $MB --steps 4 --warmup 5 --host-act-cache --act-cache-policy plan --act-cache-spill-overlap 0.8 > $O/plan_${S}_mb${MB}.log 2>&1
  run timeout -k 10 300 python -u bench.py --seq $S --micro-batch $MB --steps 3 --warmup 3 --host-act-cache --act-cache-policy ckpt_offload --act-cache-host-gib 0.01 > $O/ckstash_nospill_${S}_mb${MB}.log 2>&1
done
exit 0
