# GPU: Llama-3-8B mb10 with ZeRO-Offload Twin-Flow (offload_optimizer.ratio < 1, compact device part) against full ZeRO-Offload
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5as
mkdir -p $O
export HDS_BENCH_PROGRESS=1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload cpu"
for r in 1.0 0.6 0.5 0.4; do
  timeout -k 10 330 $B --offload-ratio $r > $O/mb10_zero_offload_ratio_$r.log 2>&1
  rc=$?; echo "ratio $r rc=$rc" >> $O/status.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
done
grep -h metric $O/*.log
