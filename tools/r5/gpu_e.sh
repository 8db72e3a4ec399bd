# GPU: where HBM genuinely runs out at the DEFAULT budget -- 32k x micro-batch 2 and 64k x micro-batch 1 -- with the
# per-tensor plan, plain activation checkpointing and ckpt_offload (verdict r4 item 2)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
export HDS_BENCH_PROGRESS=1
for shape in "32768 2" "65536 1"; do
  set -- $shape
  S=$1; MB=$2
  run timeout -k 10 420 python -u bench.py --seq $S --micro-batch $MB --steps 4 --warmup 5 --host-act-cache --act-cache-policy plan --act-cache-spill-overlap 0.8 > $O/plan_${S}_mb${MB}.log 2>&1
  run timeout -k 10 300 python -u bench.py --seq $S --micro-batch $MB --steps 3 --warmup 2 --ckpt > $O/ckpt_${S}_mb${MB}.log 2>&1
  run timeout -k 10 300 python -u bench.py --seq $S --micro-batch $MB --steps 3 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > $O/ckoff_${S}_mb${MB}.log 2>&1
done
exit 0
