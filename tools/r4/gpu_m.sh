# GPU: longest contexts with the budget-aware attention stash: 320k and 128k ckpt_offload
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4m/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
export HDS_BENCH_PROGRESS=1
run timeout -k 10 700 python -u bench.py --seq 327680 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload > gpurun_out/r4m/ckoff320k.log 2>&1
run timeout -k 10 400 python -u bench.py --seq 131072 --micro-batch 1 --steps 2 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > gpurun_out/r4m/ckoff128k.log 2>&1
