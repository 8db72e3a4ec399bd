# GPU: full gpu test suite, then functional bench runs of the secondary configs
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests2.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/gpu_tests2.log; exit 1; }
timeout -k 10 300 python bench.py --model gpt2-small --seq 1024 --micro-batch 16 --zero 1 --steps 4 --warmup 2 > gpurun_out/bench_gpt2.log 2>&1 && \
timeout -k 10 300 python bench.py --model tiny-moe --seq 1024 --micro-batch 8 --zero 3 --steps 4 --warmup 2 > gpurun_out/bench_tinymoe.log 2>&1 && \
timeout -k 10 600 python bench.py --layers 8 --offload cpu --offload-param --steps 2 --warmup 1 --micro-batch 2 > gpurun_out/bench_infinity.log 2>&1 && \
timeout -k 10 600 python bench.py --layers 8 --host-act-cache --seq 32768 --micro-batch 1 --steps 2 --warmup 1 > gpurun_out/bench_actcache32k.log 2>&1
echo "rc=$?" >> gpurun_out/bench_actcache32k.log
