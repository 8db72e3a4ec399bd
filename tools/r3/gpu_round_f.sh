# GPU: FA forward variants 5/6 parity (bisection of the DMA fast path), then round D (v2 decode diag, act cache, param offload)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rf
T="python -u -m pytest -v --timeout 150 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "staggered_variant" > gpurun_out/rf/fa_var_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/r3/gpu_round_d.sh
