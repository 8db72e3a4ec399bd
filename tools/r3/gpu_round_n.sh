# GPU (re-entry): FA backward XOR-on-base verification, transpose v2 + LM-head transposed-weight cache, batched
# split-K wgrad candidates (micro-benchmark), smoke, headline bench, 32k recompute policy
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rn
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_wgrad_layout_gpu.py > gpurun_out/rn/wgrad_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/r3/bench_transpose.py > gpurun_out/rn/transpose_bench.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_wgrad_layout.py --splitk > gpurun_out/rn/wgrad_b2.log 2>&1 || exit 1
timeout -k 10 300 $T tests/test_kernels_gpu.py tests/test_grad_parity_gpu.py -k "flash or attn or evoformer or parity" > gpurun_out/rn/flash_tests.log 2>&1 || exit 1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/rn/smoke.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rn/fa_bench.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rn/bench.log 2>&1 || exit 1
HDS_WGRAD_B2=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rn/bench_b2.log 2>&1 || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 4"
timeout -k 10 500 $B --host-act-cache --act-cache-policy recompute --act-cache-budget-gib 230 > gpurun_out/rn/ac32k_b230_recompute.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rn/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/rn/prof_bench.log 2>&1 || exit 1
python tools/r3/glue_census.py gpurun_out/rn/prof > gpurun_out/rn/glue_census.txt 2>&1
python tools/r3/trace_step_stats.py gpurun_out/rn/prof > gpurun_out/rn/step_stats.txt 2>&1
find gpurun_out/rn/prof -name "*kernel_trace.csv" -size +20M -delete
