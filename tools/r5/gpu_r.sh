# GPU: mb10 chunked optimizer-state offload vs ZeRO-Offload with the expandable-segments allocator (allocation
# retries near a full device), plus ratio 0.4
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.4 > $O/mb10_offstates_0.4.log 2>&1
export PYTORCH_HIP_ALLOC_CONF=expandable_segments:True
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.35 > $O/mb10_offstates_0.35_exp.log 2>&1
run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio 0.3 > $O/mb10_offstates_0.3_exp.log 2>&1
run timeout -k 10 300 $B --offload cpu > $O/mb10_zero_offload_exp.log 2>&1
exit 0
