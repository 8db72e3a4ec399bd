# GPU: norm kernel tests + RMSNorm backward bandwidth vs workgroup cap
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "norm" --timeout 200 --timeout-method thread > gpurun_out/norm_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_norm_bwd.py > gpurun_out/norm_bwd_bench.jsonl 2> gpurun_out/norm_bwd_bench.err || exit 1
