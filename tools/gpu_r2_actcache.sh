# GPU: 32k host activation cache after the prefetch fix, plus a kernel + memory-copy trace of it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/actc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_host_tier_gpu.py > gpurun_out/actc/test.log 2>&1 || { echo "rc=$?" >> gpurun_out/actc/test.log; exit 1; }
timeout -k 10 500 python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --steps 3 --warmup 2 > gpurun_out/actc/bench.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/actc/trace -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --steps 1 --warmup 2 > gpurun_out/actc/trace.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/actc/trace > gpurun_out/actc/overlap.txt 2>&1 || true
find gpurun_out/actc/trace -name "*.csv" -size +30M -delete
