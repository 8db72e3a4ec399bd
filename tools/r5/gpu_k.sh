# GPU: forward variants 9 / 10 (one wave per SIMD, flash_attn_w64.hip) parity against variant 2 + fp32, TF/s vs 5;
# then mb10 byte-granular optimizer-state offload at ratios that fit beside mb10 activations
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and (9 or 10)" > $O/parity.log 2>&1 || exit 1
run timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,9,10,5,9,10 x > $O/tfs.log 2>&1 || exit 1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
for r in 0.45 0.6; do
  run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio $r > $O/mb10_offstates_$r.log 2>&1
done
exit 0
