# GPU: decode tests (KV append, graph parity) + generation throughput + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_dec3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode or gemv or kv_append" --timeout 120 --timeout-method thread > gpurun_out/decode3_tests.log 2>&1 || exit 1
PYTHONPATH=. timeout -k 10 400 python -u tools/bench_decode_graph.py > gpurun_out/decode_graph_bench4.jsonl 2> gpurun_out/decode_graph_bench4.err || exit 1
PYTHONPATH=. timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec3 -o dec -- python3 tools/bench_decode_graph.py > gpurun_out/prof_dec3.log 2>&1 || exit 1
find gpurun_out/prof_dec3 -name "*kernel_trace.csv" -size +20M -delete
