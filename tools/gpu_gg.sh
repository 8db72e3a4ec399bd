# GPU: grouped GEMM numerics + micro-benchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true
timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/gg_bench.log 2>&1
