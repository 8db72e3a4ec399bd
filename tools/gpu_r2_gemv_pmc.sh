# GPU: PMC pass over the GEMV benchmark -- bytes fetched from HBM per dispatch (FETCH_SIZE) next to kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gemv
PYTHONPATH=. timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_gemv -o g -- python3 tools/bench_gemv.py > gpurun_out/pmc_gemv.log 2>&1 || exit 1
