# GPU test suite + smoke + headline bench on one MI355X (round 6). Usage: bash tools/r6/gpu_suite_bench.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r6}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/gpu_suite.log 2>&1 || { echo "suite failed rc=$?"; tail -30 gpurun_out/$TAG/gpu_suite.log; exit 1; }
tail -2 gpurun_out/$TAG/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench failed; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
