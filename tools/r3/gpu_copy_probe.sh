# GPU: copy-engine probe (SDMA vs blit kernels for side-stream D2H / H2D beside GEMMs) + its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cp
timeout -k 10 180 python -u tools/r3/copy_engine_probe.py > gpurun_out/cp/probe.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/cp/trace -o run -- python3 tools/r3/copy_engine_probe.py > gpurun_out/cp/probe_traced.log 2>&1 || exit 1
HSA_ENABLE_SDMA=1 timeout -k 10 180 python -u tools/r3/copy_engine_probe.py > gpurun_out/cp/probe_sdma1.log 2>&1 || exit 1
find gpurun_out/cp -name "*.csv" -size +20M -delete
