# GPU: decode GEMV benchmark + parity tests, decode-graph tests and Llama-3-8B generation throughput with the GEMV
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 200 python -u tools/bench_gemv.py > gpurun_out/gemv_bench.jsonl 2> gpurun_out/gemv_bench.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemv or decode" --timeout 120 --timeout-method thread > gpurun_out/gemv_tests.log 2>&1 || exit 1
PYTHONPATH=. timeout -k 10 400 python -u tools/bench_decode_graph.py > gpurun_out/decode_graph_bench_gemv.jsonl 2> gpurun_out/decode_graph_bench_gemv.err || exit 1
