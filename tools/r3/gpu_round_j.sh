# GPU: v2 decode GEMV-rule A/B, then the whole GPU test suite and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rj
timeout -k 10 200 python -u tools/r3/v2_decode_diag.py 1:graph,8:graph > gpurun_out/rj/v2_gemv_default.jsonl 2>&1 || exit 1
HDS_GEMV_MAX_NUMEL=629145600 timeout -k 10 200 python -u tools/r3/v2_decode_diag.py 1:graph,8:graph > gpurun_out/rj/v2_gemv_all.jsonl 2>&1 || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/rj/gpu_suite.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rj/smoke.log 2>&1 || exit 1
