set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_evoformer_gpu.py tests/test_kernels_gpu.py -k "evoformer or flash or attn" > gpurun_out/evo_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/evo_test.log; exit 1; }
timeout -k 10 300 python -u tools/bench_evoformer.py > gpurun_out/evo_bench.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_decode.py > gpurun_out/decode_bench.log 2>&1 || exit 1
