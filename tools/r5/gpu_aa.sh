# GPU: mb10 optimizer-state offload, one bulk reload during the one-rank backward at lower HBM fractions
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5aa
mkdir -p $O
B="python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states --offload-states-ratio 0.35"
export HDS_STATE_RELOAD_IN_BWD=1
for f in 0.85 0.8; do
  HDS_STATE_RELOAD_FRACTION=$f timeout -k 10 300 $B > $O/mb10_bwdreload_$f.log 2>&1
  echo "rc=$? $f" >> $O/status.txt
done
exit 0
