# GPU: Ulysses SP=2 device path (two ranks on one MI355X, host-staged all-to-alls)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4w
timeout -k 10 400 python -u -m pytest tests/test_sp_device_multirank_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4w/tests.log 2>&1
echo "rc=$?" >> gpurun_out/r4w/status.txt
