# GPU: ZeRO-Offload host-step piece size (sub_group_size 1e9 default vs 1e8 / 2.5e8) at mb10, Twin-Flow 0.4 and full
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ay
mkdir -p $O
export HDS_BENCH_PROGRESS=1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload cpu"
run() {
  name=$1; shift
  timeout -k 10 330 $B "$@" > $O/mb10_$name.log 2>&1
  rc=$?; echo "$name rc=$rc" >> $O/status.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
}
run twin0.4_sub1e9 --offload-ratio 0.4
run twin0.4_sub1e8 --offload-ratio 0.4 --sub-group-size 100000000
run full_sub1e8 --sub-group-size 100000000
run twin0.4_sub2.5e8 --offload-ratio 0.4 --sub-group-size 250000000
grep -h metric $O/*.log
