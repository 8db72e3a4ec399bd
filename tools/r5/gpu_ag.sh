# GPU: what block A of the one-wave forward spends: stamps of 12, 15 (no VALU slots in block A), 17 (S accumulators in AGPRs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ah
mkdir -p $O
for v in 12 15 17; do
  timeout -k 10 200 python -u tools/fa_stamps.py $v > $O/stamps_$v.log 2>&1 || exit 1
done
cat $O/stamps_*.log
