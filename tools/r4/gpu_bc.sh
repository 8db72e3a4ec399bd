# GPU: 32k activation plan vs recompute, HCache FP8, optimizer-state offload at mb10, fail-loud symmetric memory
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b gpurun_out/r4c
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4b/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230"
run timeout -k 10 300 $B --act-cache-policy plan --act-cache-spill-overlap 0.8 > gpurun_out/r4b/plan06.log 2>&1
run timeout -k 10 300 $B --act-cache-policy plan --act-cache-spill-overlap 0.8 --act-cache-spill-cost 0.2 > gpurun_out/r4b/plan02.log 2>&1
run timeout -k 10 300 $B --act-cache-policy recompute > gpurun_out/r4b/recompute.log 2>&1
run timeout -k 10 300 python -u -m pytest tests/test_inference_v2.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4c/v2_tests.log 2>&1
run timeout -k 10 300 python -u tools/bench_hcache.py --seqs 8 --ctx 2048 > gpurun_out/r4c/hcache.log 2>&1
M="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run timeout -k 10 300 $M --offload-opt-states --offload-states-ratio 0.67 > gpurun_out/r4c/mb10_offstates067.log 2>&1
run timeout -k 10 300 $M --offload cpu > gpurun_out/r4c/mb10_zero_offload_cpu.log 2>&1
run timeout -k 10 400 python -u -m pytest tests/test_symmetric_gpu.py tests/test_zero_device_multirank_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4b/symm_tests.log 2>&1
