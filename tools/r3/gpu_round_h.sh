# GPU: split-K paged decode (kernel parity, family parity, v2 decode speed), headline A/B of the FA forward variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rh
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "paged" > gpurun_out/rh/paged_tests.log 2>&1 || exit 1
timeout -k 10 400 $T tests/test_inference_v2_families.py tests/test_inference_v2.py -m gpu > gpurun_out/rh/v2_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/r3/v2_decode_diag.py > gpurun_out/rh/v2_diag.jsonl 2> gpurun_out/rh/v2_diag.err || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rh/bench_fwd2.log 2>&1 || exit 1
HDS_ATTN_FWD_VAR=5 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rh/bench_fwd5.log 2>&1 || exit 1
