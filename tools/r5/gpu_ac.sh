# GPU: where block A's cycles go -- stamps of variant 12 and its timing-only diagnostics 13 (no exp) / 14 (DMA in B)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ac
mkdir -p $O
for v in 12 13 14; do
  timeout -k 10 200 python -u tools/fa_stamps.py $v > $O/stamps_$v.log 2>&1 || exit 1
done
cat $O/stamps_*.log
