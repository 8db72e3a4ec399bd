# GPU: full GPU test suite, smoke, headline bench (round-3 end state) + kernel profile of the step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ru
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/ru/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/ru/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ru/bench.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ru/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/ru/prof_bench.log 2>&1 || exit 1
python tools/r3/glue_census.py gpurun_out/ru/prof > gpurun_out/ru/glue_census.txt 2>&1
python tools/r3/trace_step_stats.py gpurun_out/ru/prof > gpurun_out/ru/step_stats.txt 2>&1
find gpurun_out/ru/prof -name "*kernel_trace.csv" -size +20M -delete
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 4"
timeout -k 10 500 $B --host-act-cache > gpurun_out/ru/ac32k.log 2>&1 || exit 1
timeout -k 10 500 $B --host-act-cache --act-cache-policy recompute > gpurun_out/ru/ac32k_recompute.log 2>&1 || exit 1
timeout -k 10 500 $B --ckpt > gpurun_out/ru/ckpt32k.log 2>&1 || exit 1
