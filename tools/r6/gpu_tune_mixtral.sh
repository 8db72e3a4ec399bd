# Add the Mixtral-8x7B (8 layers, mb4) GEMM signatures to the TunableOp table: the Llama signatures stay (TunableOp
# loads the file and only tunes GEMMs missing from it). The table is copied to gpurun_out/r6tune_mx/ for review; the
# A/B is a separate call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6tune_mx
mkdir -p $O
for i in 1 2 3 4 5 6 7; do rm -f tuning/tunableop_results$i.csv; done  # one device: keep the tuner on file 0 only
( while true; do date >> $O/heartbeat.txt; wc -l tuning/tunableop_results0.csv >> $O/heartbeat.txt 2>/dev/null; sleep 30; done ) &
HB=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=tuning/tunableop_results%d.csv PYTORCH_TUNABLEOP_TUNING=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10 HDS_TUNABLEOP=0 \
  timeout -k 10 1050 python bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 1 --warmup 1 > $O/tune_run.log 2>&1
rc=$?
kill $HB 2>/dev/null
cp tuning/tunableop_results0.csv $O/ 2>/dev/null
echo "tune rc=$rc"
wc -l tuning/tunableop_results0.csv
