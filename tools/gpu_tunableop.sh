# Tune every GEMM shape of the bench with PyTorch TunableOp (hipBLASLt + rocBLAS candidates), then
# re-run the bench reading the tuned table.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_TUNING=1
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100
export PYTORCH_TUNABLEOP_VERBOSE=1
timeout -k 10 900 python bench.py --steps 1 --warmup 1 > gpurun_out/tune/tune_run.log 2>&1 || exit 1
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 600 python bench.py --steps 6 --warmup 3 > gpurun_out/tune/bench_tuned.log 2>&1
