# GPU: inference-v2 ragged decode throughput with / without the decode GEMV (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HDS_GEMV_MAX_NUMEL=0 timeout -k 10 400 python -u tools/bench_v2_decode.py > gpurun_out/v2_decode_off.jsonl 2> gpurun_out/v2_decode_off.err || exit 1
timeout -k 10 400 python -u tools/bench_v2_decode.py > gpurun_out/v2_decode_on.jsonl 2> gpurun_out/v2_decode_on.err || exit 1
