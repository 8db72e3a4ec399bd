set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "attn or attention or quant" > gpurun_out/kt_attn.log 2>&1 && \
timeout -k 10 300 python tools/bench_attn.py > gpurun_out/attn_bench2.log 2>&1
echo "rc=$?" >> gpurun_out/attn_bench2.log
