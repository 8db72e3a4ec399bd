# GPU: round-2 re-verification (gpu suite + smoke + default bench + rocprof kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r2.log 2>&1 || { echo "tests rc=$?" >> gpurun_out/gpu_tests_r2.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r2.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_r2.log 2>&1 || exit 1
bash tools/gpu_profile.sh
