# GPU: pipeline PP=2 on the device path (two stages on one MI355X, host-staged p2p)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4u
timeout -k 10 500 python -u -m pytest tests/test_pipe_device_multirank_gpu.py tests/test_kernels_gpu.py -k "pipeline or adam" -v --timeout 300 --timeout-method thread > gpurun_out/r4u/tests.log 2>&1
echo "rc=$?" >> gpurun_out/r4u/status.txt
