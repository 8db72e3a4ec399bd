# GPU (re-entry): verify FA backward XOR-on-base on the GPU, smoke, headline bench, 32k recompute policy
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rm
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py tests/test_grad_parity_gpu.py -k "flash or attn or evoformer or parity" > gpurun_out/rm/flash_tests.log 2>&1 || exit 1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/rm/smoke.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/r3/fa_bench.py > gpurun_out/rm/fa_bench.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rm/bench.log 2>&1 || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 4"
timeout -k 10 500 $B --host-act-cache --act-cache-policy recompute --act-cache-budget-gib 230 > gpurun_out/rm/ac32k_b230_recompute.log 2>&1 || exit 1
timeout -k 10 500 $B --host-act-cache --act-cache-policy recompute --act-cache-budget-gib 200 > gpurun_out/rm/ac32k_b200_recompute.log 2>&1 || exit 1
