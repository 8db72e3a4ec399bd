# GPU: v2 decode graphs (tests + throughput), 32k host activation cache with the copy window, optimizer-state
# offload vs ZeRO-Offload CPU Adam at the headline shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rb
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_inference_v2.py -m gpu > gpurun_out/rb/v2_tests.log 2>&1
rc=$?; echo "v2 tests rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_v2_decode.py > gpurun_out/rb/v2_decode.jsonl 2> gpurun_out/rb/v2_decode.err || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 3 --warmup 2"
timeout -k 10 400 $B --host-act-cache > gpurun_out/rb/ac32k.log 2>&1 || exit 1
timeout -k 10 400 $B --host-act-cache --act-cache-budget-gib 230 > gpurun_out/rb/ac32k_b230.log 2>&1 || exit 1
timeout -k 10 400 $B --host-act-cache --act-cache-budget-gib 215 > gpurun_out/rb/ac32k_b215.log 2>&1 || exit 1
timeout -k 10 400 $B --ckpt > gpurun_out/rb/ckpt32k.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --offload-opt-states > gpurun_out/rb/oos_mb7.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --offload cpu > gpurun_out/rb/zoff_mb7.log 2>&1 || exit 1
