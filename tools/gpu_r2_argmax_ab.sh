# GPU: same-box A/B of the chunked greedy argmax in Llama-3-8B generation (3 alternating runs each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  HDS_CHUNKED_ARGMAX=0 PYTHONPATH=. timeout -k 10 300 python -u tools/bench_decode_graph.py >> gpurun_out/argmax_ab_off.jsonl 2>/dev/null || exit 1
  HDS_CHUNKED_ARGMAX=1 PYTHONPATH=. timeout -k 10 300 python -u tools/bench_decode_graph.py >> gpurun_out/argmax_ab_on.jsonl 2>/dev/null || exit 1
done
