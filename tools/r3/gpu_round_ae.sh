# GPU: copy/compute overlap traces (rocprofv3 kernel + memory-copy trace) of the ckpt_offload policy at 128k and the
# auto policy at 32k / 230 GiB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rae
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/rae/ckoff128k -o run -- python3 bench.py --seq 131072 --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload --steps 1 --warmup 1 > gpurun_out/rae/ckoff128k.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/rae/ckoff128k > gpurun_out/rae/overlap_ckoff128k.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/rae/auto32k -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy auto --act-cache-budget-gib 230 --steps 1 --warmup 5 > gpurun_out/rae/auto32k.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/rae/auto32k > gpurun_out/rae/overlap_auto32k.txt 2>&1 || true
find gpurun_out/rae -name "*.csv" -size +20M -delete
