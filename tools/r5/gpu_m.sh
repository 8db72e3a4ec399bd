# GPU: SQ counters of the FlashAttention forward variants 5 (8-wave software-pipelined) and 10 (one wave per SIMD,
# rebalanced) at the bench shape
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
for v in 5 10; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $O/p1_$v -o run -- python3 tools/fa_fwd_only.py $v > $O/p1_$v.log 2>&1 || exit 1
  python3 tools/r3/pmc_dump.py $O/p1_$v > $O/p1_$v.txt 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p2_$v -o run -- python3 tools/fa_fwd_only.py $v > $O/p2_$v.log 2>&1 || exit 1
  python3 tools/r3/pmc_dump.py $O/p2_$v > $O/p2_$v.txt 2>&1
done
find $O -name "*.csv" -size +20M -delete
cat $O/p*_*.txt
