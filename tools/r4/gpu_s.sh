# GPU: expert parallelism EP=2 on the device path (two ranks on one MI355X, host-staged all-to-all)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4s
timeout -k 10 400 python -u -m pytest tests/test_moe_device_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4s/tests.log 2>&1
echo "rc=$?" >> gpurun_out/r4s/status.txt
