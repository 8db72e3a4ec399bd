# GPU: the round-3 GPU tests (full-step gradient parity, world-2 device path, decode attention with lens/window),
# then the 32k act-cache A/B vs the last good commit with traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/acb
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_grad_parity_gpu.py tests/test_zero_device_multirank_gpu.py "tests/test_kernels_gpu.py::test_decode_attention_matches_reference_gpu" -s > gpurun_out/acb/newtests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/r3/gpu_actcache_bisect.sh
