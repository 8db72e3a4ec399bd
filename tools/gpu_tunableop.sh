# Tune every GEMM shape of the bench with PyTorch TunableOp (hipBLASLt + rocBLAS candidates). Results accumulate
# in tuning/tunableop_results0.csv (already-tuned shapes are skipped), so the tuning can span several calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune tuning
( while true; do date >> gpurun_out/tune/heartbeat.txt; wc -l tuning/tunableop_results0.csv >> gpurun_out/tune/heartbeat.txt 2>/dev/null; sleep 45; done ) &
HB=$!
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME=tuning/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30
export PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
timeout -k 10 ${TUNE_SECONDS:-1000} python bench.py --steps 1 --warmup 1 > gpurun_out/tune/tune_run.log 2>&1
rc=$?
cp tuning/tunableop_results0.csv gpurun_out/tune/tunableop_results0.csv
kill $HB 2>/dev/null
exit $rc
