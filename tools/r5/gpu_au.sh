# GPU: offload_adam_states with host-step tails (host Adam on the byte-granular tails): GPU test + mb10 against
# ZeRO-Offload on the same box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5av
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_host_tier_gpu.py -k "host_step or chunked_state_offload or twin_flow" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
export HDS_BENCH_PROGRESS=1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run() {
  name=$1; shift
  timeout -k 10 330 $B "$@" > $O/mb10_$name.log 2>&1
  rc=$?; echo "$name rc=$rc" >> $O/status.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run offstates_hoststep_0.4 --offload-opt-states --offload-states-ratio 0.4 --offload-states-host-step
run offstates_hoststep_0.5 --offload-opt-states --offload-states-ratio 0.5 --offload-states-host-step
run zero_offload --offload cpu
run offstates_hoststep_0.35 --offload-opt-states --offload-states-ratio 0.35 --offload-states-host-step
grep -h metric $O/*.log
