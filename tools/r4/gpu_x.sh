# GPU: init_inference AutoTP=2 + kernel injection on the device path (two ranks on one MI355X)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4x
timeout -k 10 400 python -u -m pytest tests/test_inference_tp_device_multirank_gpu.py tests/test_inference_v2_tp_device_multirank_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4x/tests.log 2>&1
echo "rc=$?" >> gpurun_out/r4x/status.txt
