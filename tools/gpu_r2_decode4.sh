# GPU: decode tests + generation throughput after the chunked argmax
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode or gemv or kv_append or argmax" --timeout 120 --timeout-method thread > gpurun_out/decode4_tests.log 2>&1 || exit 1
PYTHONPATH=. timeout -k 10 400 python -u tools/bench_decode_graph.py > gpurun_out/decode_graph_bench5.jsonl 2> gpurun_out/decode_graph_bench5.err || exit 1
