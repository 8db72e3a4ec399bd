# GEMM evidence (round 6): per-shape census of one headline step + a PMC pass over hipBLASLt at the bench shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6gemm
timeout -k 10 400 python tools/r6/gemm_shape_census.py gpurun_out/r6gemm/census.jsonl > gpurun_out/r6gemm/census.txt 2>&1 || { echo census failed; tail -20 gpurun_out/r6gemm/census.txt; exit 1; }
head -60 gpurun_out/r6gemm/census.txt
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --stats --output-format csv -d gpurun_out/r6gemm/pmc -o pmc -- python3 tools/r6/gemm_pmc.py > gpurun_out/r6gemm/pmc_run.txt 2>&1 || { echo pmc failed; tail -20 gpurun_out/r6gemm/pmc_run.txt; exit 1; }
grep tflops gpurun_out/r6gemm/pmc_run.txt
find gpurun_out/r6gemm/pmc -name "*.csv" | head
