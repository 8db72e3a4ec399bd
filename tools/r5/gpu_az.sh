# GPU: ZeRO-Offload at mb10 with the capped pipeline piece (defaults): Twin-Flow 0.4 and full offload, same box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5az
mkdir -p $O
export HDS_BENCH_PROGRESS=1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
run() {
  name=$1; shift
  timeout -k 10 330 $B "$@" > $O/mb10_$name.log 2>&1
  rc=$?; echo "$name rc=$rc" >> $O/status.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run twin0.4 --offload cpu --offload-ratio 0.4
run zero_offload --offload cpu
run offstates_hoststep_0.35 --offload-opt-states --offload-states-ratio 0.35 --offload-states-host-step
grep -h metric $O/*.log
