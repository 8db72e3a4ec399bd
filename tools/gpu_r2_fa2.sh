set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fapmc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "staggered or flash" > gpurun_out/fa_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/fa_test.log; exit 1; }
timeout -k 10 300 python -u tools/bench_attn_fwd_variants.py > gpurun_out/fa_bench.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 -L > gpurun_out/fapmc/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --kernel-trace -d gpurun_out/fapmc/p1 -o run --output-format csv -- python tools/fa_fwd_only.py 2 > gpurun_out/fapmc/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/fapmc/p2 -o run --output-format csv -- python tools/fa_fwd_only.py 2 > gpurun_out/fapmc/p2.log 2>&1 || exit 1
