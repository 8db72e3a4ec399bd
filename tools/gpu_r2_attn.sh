# GPU: head-dim generic attention kernels (FA fwd/bwd, paged, RoPE scatter), BERT/GPT-2/serving families, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "flash or paged or rope or qkv" > gpurun_out/attn_tests_r2.log 2>&1 || { echo "rc=$?" >> gpurun_out/attn_tests_r2.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_transformer_layer.py tests/test_gpt2_gpu.py tests/test_inference_v2_families.py > gpurun_out/attn_models_r2.log 2>&1 || { echo "rc=$?" >> gpurun_out/attn_models_r2.log; exit 1; }
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_r2_attn.log 2>&1
