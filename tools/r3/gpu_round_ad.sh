# GPU: multi-rank ZeRO-3 device-path tests (comm stats with real Work objects) after the comm-stats retention fix
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rad
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_zero_device_multirank_gpu.py tests/test_symmetric_gpu.py > gpurun_out/rad/multirank_tests.log 2>&1 || exit 1
