# GPU: AutoTP = 2 on the device path (two ranks on one MI355X, symmetric one-shot forward all-reduces)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4t
timeout -k 10 400 python -u -m pytest tests/test_tp_device_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4t/tests.log 2>&1
echo "rc=$?" >> gpurun_out/r4t/status.txt
