# GPU: attention epilogue stores widened to 16 B (permlane32 pairs) -- parity tests, A/B against the 8-B stores
# (HDS_KERNEL_LIB A/B library from tools/r4/build_ab_narrow.py), headline bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4j
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4j/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash or paged" -x -v --timeout 120 --timeout-method thread > gpurun_out/r4j/fa_tests.log 2>&1 || exit 1
N=hcache_deepspeed_amd/_lib/libhds_kernels_narrow.so
W=hcache_deepspeed_amd/_lib/libhds_kernels.so
for L in $N $W $N $W; do
  echo "== $L" >> gpurun_out/r4j/ab.log
  HDS_KERNEL_LIB=$L run timeout -k 10 200 python -u tools/bench_attn_fwd_variants.py 5,5 >> gpurun_out/r4j/ab.log 2>&1 || exit 1
done
run timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4j/bench.log 2>&1
