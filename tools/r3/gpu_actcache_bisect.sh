# GPU: 32k host activation cache, 230 GiB budget: same-box A/B of the last good commit (9b92f67) vs HEAD, and a
# kernel + memory-copy trace of HEAD's step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/acb
B="bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-budget-gib 230 --warmup 2"
(cd _bisect/good && timeout -k 10 400 python -u $B --steps 3) > gpurun_out/acb/good_b230.log 2>&1 || exit 1
timeout -k 10 400 python -u $B --steps 3 > gpurun_out/acb/head_b230.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/acb/trace_head -o run -- python3 $B --steps 1 > gpurun_out/acb/trace_head.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/acb/trace_head > gpurun_out/acb/overlap_head.txt 2>&1 || true
python3 tools/r3/trace_step_stats.py gpurun_out/acb/trace_head > gpurun_out/acb/stats_head.txt 2>&1 || true
(cd _bisect/good && timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d ../../gpurun_out/acb/trace_good -o run -- python3 $B --steps 1) > gpurun_out/acb/trace_good.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/acb/trace_good > gpurun_out/acb/overlap_good.txt 2>&1 || true
python3 tools/r3/trace_step_stats.py gpurun_out/acb/trace_good > gpurun_out/acb/stats_good.txt 2>&1 || true
find gpurun_out/acb -name "*.csv" -size +20M -delete
