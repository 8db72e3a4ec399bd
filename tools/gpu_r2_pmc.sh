# GPU: MFMA utilisation of the training step's kernels (Llama-3-8B width, 2 layers, mb7; counters serialise
# dispatches, so a short run) -- PMC pass in its own run with --kernel-trace only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc/step -o run -- python3 bench.py --layers 2 --steps 1 --warmup 1 > gpurun_out/pmc/step.log 2>&1 || { echo "pmc rc=$?" >> gpurun_out/pmc/step.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc/step gpurun_out/pmc/mfma_util.txt > /dev/null
find gpurun_out/pmc -name "*.csv" -size +20M -delete
