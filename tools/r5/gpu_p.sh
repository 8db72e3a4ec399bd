# GPU: forward variants 10/11 parity + TF/s vs 5; mb10 chunked optimizer-state offload; SQ counters of 5/10/11
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "staggered_variant and (10 or 11)" > $O/parity.log 2>&1 || exit 1
run timeout -k 10 240 python -u tools/bench_attn_fwd_variants.py 5,10,11,5,10,11,5,11 x > $O/tfs.log 2>&1 || exit 1
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3"
for r in 0.35 0.45; do
  run timeout -k 10 300 $B --offload-opt-states --offload-states-ratio $r > $O/mb10_offstates_$r.log 2>&1
done
cat $O/tfs.log
P=gpurun_out/r5m
mkdir -p $P
for v in 5 10 11; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $P/p1_$v -o run -- python3 tools/fa_fwd_only.py $v > $P/p1_$v.log 2>&1 || exit 1
  python3 tools/r3/pmc_dump.py $P/p1_$v > $P/p1_$v.txt 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $P/p2_$v -o run -- python3 tools/fa_fwd_only.py $v > $P/p2_$v.log 2>&1 || exit 1
  python3 tools/r3/pmc_dump.py $P/p2_$v > $P/p2_$v.txt 2>&1
done
find $P -name "*.csv" -size +20M -delete
cat $P/p*_*.txt
exit 0
