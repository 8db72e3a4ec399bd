# TunableOp over every GEMM signature of the headline step (hipBLASLt + rocBLAS candidates), then the headline bench
# with and without the table on the same box (round 6; round 1 found no gain with the libraries of then)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6tune
mkdir -p $O tuning
rm -f tuning/tunableop_results0.csv
( while true; do date >> $O/heartbeat.txt; wc -l tuning/tunableop_results0.csv >> $O/heartbeat.txt 2>/dev/null; sleep 30; done ) &
HB=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=tuning/tunableop_results%d.csv PYTORCH_TUNABLEOP_TUNING=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10 \
  timeout -k 10 600 python bench.py --steps 1 --warmup 1 > $O/tune_run.log 2>&1
rc=$?
kill $HB 2>/dev/null
cp tuning/tunableop_results0.csv $O/ 2>/dev/null
[ $rc -eq 0 ] || { echo "tune rc=$rc"; tail -20 $O/tune_run.log; exit 1; }
wc -l tuning/tunableop_results0.csv
for t in 1 0 1 0; do
  HDS_TUNABLEOP=$t timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_tuned$t.json 2> $O/bench_tuned$t.err || { echo "bench $t failed"; tail -20 $O/bench_tuned$t.err; exit 1; }
  python -c "import json;d=json.loads([l for l in open('$O/bench_tuned$t.json') if l.startswith('{')][-1]);print('tuned=$t', d['value'], d['extra']['tuned_gemm_table'])"
done
