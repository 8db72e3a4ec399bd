# GPU: host-tier / act-plan / symmetric tests after the round-5 changes; 128k ckpt_offload with the summed boundary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 600 python -u -m pytest tests/test_host_tier_gpu.py tests/test_act_plan_gpu.py tests/test_symmetric_gpu.py tests/test_zero_device_multirank_gpu.py -x -v --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || exit 1
export HDS_BENCH_PROGRESS=1
run timeout -k 10 400 python -u bench.py --seq 131072 --micro-batch 1 --steps 3 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > $O/ckoff128k.log 2>&1
exit 0
