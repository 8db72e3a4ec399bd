# rocprofv3 kernel-trace + stats of a short full-model bench run (1 GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/prof_bench.log
find gpurun_out/prof -name "*kernel_stats.csv" | head -5 >> gpurun_out/prof_bench.log
# drop the big per-dispatch trace to stay under the merge cap
find gpurun_out/prof -name "*kernel_trace.csv" -size +20M -delete
exit $rc
