# GPU: HIP-graph decode tests + Llama-3-8B generation throughput eager vs graph
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "decode" --timeout 200 --timeout-method thread > gpurun_out/decode_graph_tests.log 2>&1 || exit 1
PYTHONPATH=. timeout -k 10 400 python -u tools/bench_decode_graph.py > gpurun_out/decode_graph_bench.jsonl 2> gpurun_out/decode_graph_bench.err || exit 1
