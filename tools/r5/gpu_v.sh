# GPU: forward variants 10-12 with 4 K/V slots and a barrier per tile pair (parity, stamps, timing); mb10 state offload
# with the single-allocation backward reload
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5v
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and (10 or 11)" > $O/parity.log 2>&1 || exit 1
run timeout -k 10 200 python -u tools/fa_stamps.py > $O/stamps.log 2>&1 || exit 1
run timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,11,5,11,5,11 x > $O/fwd.log 2>&1 || exit 1
cat $O/stamps.log $O/fwd.log
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.35 > $O/mb10_offstates_0.35.log 2>&1
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.4 > $O/mb10_offstates_0.4.log 2>&1
exit 0
