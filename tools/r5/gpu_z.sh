# GPU: FPDT attention at long context on one MI355X (chunked, host-offloaded q/k/v/o/lse) vs plain fused-QKV attention
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 600 python -u tools/bench_fpdt.py 65536,131072,262144 8 > $O/fpdt.jsonl 2> $O/fpdt.err
echo "rc=$?" >> $O/status.txt
cat $O/fpdt.jsonl
