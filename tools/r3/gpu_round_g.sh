# GPU: FA kernels after tying LDS-read fragments to their waits (all flash tests, variants 4/5/6, variant timing),
# then the 32k host activation cache with the closed-loop plan + budget-bounded prefetch-ahead
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rg
T="python -u -m pytest -v --timeout 150 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py -k "flash or attn" > gpurun_out/rg/flash_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_attn_fwd_variants.py > gpurun_out/rg/fa_var_bench.log 2>&1 || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 3"
timeout -k 10 500 $B --host-act-cache --act-cache-budget-gib 230 > gpurun_out/rg/ac32k_b230.log 2>&1 || exit 1
timeout -k 10 500 $B --host-act-cache > gpurun_out/rg/ac32k.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rg/v2prof -o v2 -- python3 tools/r3/v2_decode_diag.py 1:graph > gpurun_out/rg/v2prof.log 2>&1 || exit 1
find gpurun_out/rg/v2prof -name "*kernel_trace.csv" -delete
