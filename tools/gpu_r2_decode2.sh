# GPU: decode attention tests + Llama-3-8B generation throughput + kernel stats after the split change
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_dec2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode or gemv" --timeout 120 --timeout-method thread > gpurun_out/decode2_tests.log 2>&1 || exit 1
PYTHONPATH=. timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec2 -o dec -- python3 tools/bench_decode_graph.py > gpurun_out/prof_dec2.log 2>&1 || exit 1
find gpurun_out/prof_dec2 -name "*kernel_trace.csv" -size +20M -delete
PYTHONPATH=. timeout -k 10 400 python -u tools/bench_decode_graph.py > gpurun_out/decode_graph_bench3.jsonl 2> gpurun_out/decode_graph_bench3.err || exit 1
