# GPU: rocprofv3 kernel stats of the Llama-3-8B generation benchmark (HIP-graph decode + GEMV)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_dec
PYTHONPATH=. timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec -o dec -- python3 tools/bench_decode_graph.py > gpurun_out/prof_dec.log 2>&1 || exit 1
find gpurun_out/prof_dec -name "*kernel_trace.csv" -size +20M -delete
