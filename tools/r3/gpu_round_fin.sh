# GPU: end-of-session verification: full GPU test suite, smoke, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rfin
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/rfin/gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/rfin/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rfin/bench.log 2>&1 || exit 1
