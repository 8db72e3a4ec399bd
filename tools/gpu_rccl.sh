# GPU: native RCCL executor tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_rccl.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/rccl_tests.log 2>&1
echo "rc=$?" >> gpurun_out/rccl_tests.log
