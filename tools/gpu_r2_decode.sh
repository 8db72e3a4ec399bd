# GPU: decode attention kernel + v1 family generation through the KV cache
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_inference_v1_families.py tests/test_inference_v1.py -k "decode_attention or family or kernel_injection" > gpurun_out/decode_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/decode_test.log; exit 1; }
