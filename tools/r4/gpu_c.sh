# GPU: HCache FP8 latents (tests + restore bench), then optimizer-state offload where the states do not fit
# (Llama-3-8B, seq 4096, micro-batch 10: ~300 GiB with states resident) against ZeRO-Offload CPU Adam
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4c
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4c/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run timeout -k 10 300 python -u -m pytest tests/test_inference_v2.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4c/v2_tests.log 2>&1
run timeout -k 10 400 python -u tools/bench_hcache.py --seqs 8 --ctx 2048 > gpurun_out/r4c/hcache.log 2>&1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run timeout -k 10 500 $B --offload-opt-states --offload-states-ratio 0.67 > gpurun_out/r4c/mb10_offstates067.log 2>&1
run timeout -k 10 500 $B --offload-opt-states > gpurun_out/r4c/mb10_offstates100.log 2>&1
run timeout -k 10 600 $B --offload cpu > gpurun_out/r4c/mb10_zero_offload_cpu.log 2>&1
