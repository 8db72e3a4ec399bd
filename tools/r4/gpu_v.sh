# GPU: ZeRO-1/2 (+ fp32) device path at world 2 on one MI355X
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4v
timeout -k 10 600 python -u -m pytest tests/test_zero_device_multirank_gpu.py -k "zeropp" -v --timeout 300 --timeout-method thread > gpurun_out/r4v/tests.log 2>&1
echo "rc=$?" >> gpurun_out/r4v/status.txt
