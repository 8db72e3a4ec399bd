# GPU: FlashAttention at the bench shape after the widened epilogue stores: timings + one SQ counter pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4r
timeout -k 10 120 python -u tools/r3/fa_bench.py > gpurun_out/r4r/time.log 2>&1 || exit 1
P="python3 tools/r3/fa_bench.py --iters 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/r4r/p1 -o run -- $P > gpurun_out/r4r/p1.log 2>&1 || exit 1
python3 tools/r3/pmc_dump.py gpurun_out/r4r/p1 > gpurun_out/r4r/p1.txt 2>&1
find gpurun_out/r4r -name "*.csv" -size +20M -delete
