# GPU: re-verify the rebuilt tree (gpu test suite + smoke + default bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests5.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/gpu_tests5.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke5.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_r5.log 2>&1
