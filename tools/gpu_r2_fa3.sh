set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_gpt2_gpu.py -k "staggered or flash or attn or gpt2" > gpurun_out/fa_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/fa_test.log; exit 1; }
timeout -k 10 300 python -u tools/bench_attn_fwd_variants.py > gpurun_out/fa_bench.log 2>&1 || exit 1
