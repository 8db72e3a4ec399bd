# GPU: Evoformer HIP forward numerics + micro-benchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_evoformer_gpu.py tests/test_evoformer_cpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/evo_tests.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/evo_tests.log; exit 1; }
timeout -k 10 300 python -u tools/bench_evoformer.py > gpurun_out/evo_bench.log 2>&1
