# GPU: attention stash spilled (host tier tests), 320k / 128k ckpt_offload with it, 32k plan regression check
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4p/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 300 python -u -m pytest tests/test_host_tier_gpu.py tests/test_act_plan_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4p/tests.log 2>&1 || exit 1
export HDS_BENCH_PROGRESS=1
run timeout -k 10 700 python -u bench.py --seq 327680 --micro-batch 1 --steps 1 --warmup 1 --host-act-cache --act-cache-policy ckpt_offload --act-cache-host-gib 225 > gpurun_out/r4p/ckoff320k.log 2>&1
run timeout -k 10 400 python -u bench.py --seq 131072 --micro-batch 1 --steps 2 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > gpurun_out/r4p/ckoff128k.log 2>&1
run timeout -k 10 300 python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8 --steps 6 --warmup 6 > gpurun_out/r4p/plan32k.log 2>&1
exit 0
