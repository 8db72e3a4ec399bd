# GPU: full-width Mixtral-8x7B (4096 hidden, 8 experts x 14336, top-2) ZeRO-3 on 1 MI355X, reduced depth
# (a 1-GPU box cannot hold 32 layers' optimizer state: 46.7B params x 16 B; marked valid:false by bench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --model mixtral-8x7b --layers 8 --micro-batch 2 --steps 3 --warmup 1 > gpurun_out/mixtral_l8_mb2.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --model mixtral-8x7b --layers 8 --micro-batch 4 --steps 3 --warmup 1 > gpurun_out/mixtral_l8_mb4.log 2>&1 || exit 1
