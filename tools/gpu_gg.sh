# GPU: grouped GEMM micro-benchmark + one PMC pass (MFMA busy, LDS bank conflicts) on the quick shape
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_grouped_gemm.py > gpurun_out/gg_bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_gg -o run -- python3 tools/bench_grouped_gemm.py --quick > gpurun_out/pmc_gg.log 2>&1
echo "pmc rc=$?" >> gpurun_out/pmc_gg.log
