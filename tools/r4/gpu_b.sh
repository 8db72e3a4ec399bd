# GPU: fail-loud symmetric memory tests, then 32k / 230 GiB: plan (spill cost 0.6 and 0.2) vs recompute
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
run() {  # a failing test is recorded; a fault / abort / time limit ends the script
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4b/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run timeout -k 10 600 python -u -m pytest tests/test_symmetric_gpu.py tests/test_zero_device_multirank_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4b/symm_tests.log 2>&1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230"
run timeout -k 10 400 $B --act-cache-policy plan --act-cache-spill-overlap 0.8 > gpurun_out/r4b/plan06.log 2>&1
run timeout -k 10 400 $B --act-cache-policy plan --act-cache-spill-overlap 0.8 --act-cache-spill-cost 0.2 > gpurun_out/r4b/plan02.log 2>&1
run timeout -k 10 400 $B --act-cache-policy recompute > gpurun_out/r4b/recompute.log 2>&1
