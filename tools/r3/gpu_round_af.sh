# GPU: fused Adam with non-temporal stores (HDS_ADAM_NT=1) vs plain: parity test + micro-benchmark; then copy/compute
# overlap traces of ckpt_offload at 128k and the auto policy at 32k / 230 GiB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/raf
T="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
HDS_ADAM_NT=1 timeout -k 10 300 $T tests/test_kernels_gpu.py -k "adam" > gpurun_out/raf/adam_tests_nt.log 2>&1 || exit 1
for r in 1 2; do
  HDS_ADAM_NT=0 timeout -k 10 120 python -u tools/r3/bench_adam.py >> gpurun_out/raf/adam_bench.log 2>&1 || exit 1
  HDS_ADAM_NT=1 timeout -k 10 120 python -u tools/r3/bench_adam.py >> gpurun_out/raf/adam_bench.log 2>&1 || exit 1
done
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/raf/ckoff128k -o run -- python3 bench.py --seq 131072 --micro-batch 1 --host-act-cache --act-cache-policy ckpt_offload --steps 1 --warmup 1 > gpurun_out/raf/ckoff128k.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/raf/ckoff128k > gpurun_out/raf/overlap_ckoff128k.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/raf/auto32k -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy auto --act-cache-budget-gib 230 --steps 1 --warmup 5 > gpurun_out/raf/auto32k.log 2>&1 || exit 1
python3 tools/overlap_report.py gpurun_out/raf/auto32k > gpurun_out/raf/overlap_auto32k.txt 2>&1 || true
find gpurun_out/raf -name "*.csv" -size +20M -delete
