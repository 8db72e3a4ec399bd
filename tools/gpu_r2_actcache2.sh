set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HDS_BENCH_PROGRESS=1
mkdir -p gpurun_out/actc
for B in 230 200; do
  timeout -k 10 400 python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-budget-gib $B --steps 3 --warmup 2 > gpurun_out/actc/bench_b$B.log 2>&1 || exit 1
done
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/actc/trace2 -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-budget-gib 200 --steps 1 --warmup 2 > gpurun_out/actc/trace2.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/actc/trace2 > gpurun_out/actc/overlap2.txt 2>&1 || true
find gpurun_out/actc/trace2 -name "*.csv" -size +30M -delete
