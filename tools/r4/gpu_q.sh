# GPU: 128k ckpt_offload with the stash kept on the device where the HBM allows; host tier tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4q
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4q/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 300 python -u -m pytest tests/test_host_tier_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4q/tests.log 2>&1 || exit 1
export HDS_BENCH_PROGRESS=1
run timeout -k 10 500 python -u bench.py --seq 131072 --micro-batch 1 --steps 3 --warmup 2 --host-act-cache --act-cache-policy ckpt_offload > gpurun_out/r4q/ckoff128k.log 2>&1
exit 0
