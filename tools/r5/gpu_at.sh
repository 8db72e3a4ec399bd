# GPU: Twin-Flow GPU test; mb10 Twin-Flow at ratio 0.35 / 0.3
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5at
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_host_tier_gpu.py -k "twin_flow or nvme_tier" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
export HDS_BENCH_PROGRESS=1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload cpu"
for r in 0.35 0.3; do
  timeout -k 10 330 $B --offload-ratio $r > $O/mb10_zero_offload_ratio_$r.log 2>&1
  rc=$?; echo "ratio $r rc=$rc" >> $O/status.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
done
grep -h metric $O/*.log
