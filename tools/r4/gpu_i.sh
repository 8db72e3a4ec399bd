# GPU: FlashAttention forward variant 9 (one wave per SIMD, 64 query rows per wave) -- parity tests, A/B against the
# default variant 5 at the bench shape, per-kernel time
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4i/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "staggered_variant and (5 or 9)" -x -v --timeout 120 --timeout-method thread > gpurun_out/r4i/fa_tests.log 2>&1 || exit 1
run timeout -k 10 200 python -u tools/bench_attn_fwd_variants.py 5,9,5,9,9 nobwd > gpurun_out/r4i/fa_fwd_ab.log 2>&1
run timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i/prof9 -o run -- python3 tools/fa_fwd_only.py 9 > gpurun_out/r4i/prof9.log 2>&1
run timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i/prof5 -o run -- python3 tools/fa_fwd_only.py 5 > gpurun_out/r4i/prof5.log 2>&1
find gpurun_out/r4i -name "*kernel_trace.csv" -delete
exit 0
