# GPU: maximum trainable sequence length of Llama-3-8B (ZeRO-3, 1 x MI355X, 288 GB HBM), activation checkpointing,
# then + CPU optimizer offload. Each length is its own process under its own time limit; an OOM ends that arm.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HDS_BENCH_PROGRESS=1
mkdir -p gpurun_out/seq
run() {  # name, timeout, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py --micro-batch 1 "$@" > gpurun_out/seq/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/seq/summary.txt
  grep '^{' gpurun_out/seq/$name.log >> gpurun_out/seq/summary.txt
  return $rc
}
run ckpt_64k 300 --seq 65536 --ckpt --steps 1 --warmup 1 || exit 0
run ckpt_128k 420 --seq 131072 --ckpt --steps 1 --warmup 1 || exit 0
run ckpt_256k 600 --seq 262144 --ckpt --steps 1 --warmup 1 || exit 0
