# GPU: forward variant 11/12 with the LDS-DMA issued in block A (stamps + timing + parity); mb10 optimizer-state
# offload with the expandable-segments allocator (PYTORCH_ALLOC_CONF) against ZeRO-Offload under the same allocator
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 200 python -u tools/fa_stamps.py > $O/stamps.log 2>&1 || exit 1
run timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and 11" > $O/parity.log 2>&1 || exit 1
run timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,11,5,11 x > $O/fwd.log 2>&1 || exit 1
cat $O/stamps.log $O/fwd.log
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
export PYTORCH_ALLOC_CONF=expandable_segments:True
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.35 > $O/mb10_offstates_0.35_exp.log 2>&1
run timeout -k 10 300 $B --offload cpu > $O/mb10_zero_offload_exp.log 2>&1
exit 0
