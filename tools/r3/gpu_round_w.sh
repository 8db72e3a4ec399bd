# GPU: FlashAttention PMC passes on the round-3 end kernels (sp forward, PIPE 2 backward, no-SLP build); then 32k host activation cache under a 230 GiB budget, spill vs recompute
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fa2
timeout -k 10 120 python -u tools/r3/fa_bench.py > gpurun_out/fa2/time.log 2>&1 || exit 1
P="python3 tools/r3/fa_bench.py --iters 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/fa2/p1 -o run -- $P > gpurun_out/fa2/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d gpurun_out/fa2/p2 -o run -- $P > gpurun_out/fa2/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES --kernel-trace --output-format csv -d gpurun_out/fa2/p3 -o run -- $P > gpurun_out/fa2/p3.log 2>&1 || exit 1
for p in p1 p2 p3; do python3 tools/r3/pmc_dump.py gpurun_out/fa2/$p > gpurun_out/fa2/$p.txt 2>&1; done
find gpurun_out/fa2 -name "*.csv" -size +20M -delete
mkdir -p gpurun_out/rv
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 4 --host-act-cache --act-cache-budget-gib 230"
timeout -k 10 500 $B > gpurun_out/rv/ac32k_b230_spill.log 2>&1 || exit 1
timeout -k 10 500 $B --act-cache-policy recompute > gpurun_out/rv/ac32k_b230_recompute.log 2>&1 || exit 1
