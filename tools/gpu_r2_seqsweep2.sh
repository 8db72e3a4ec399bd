# GPU: long-context arms past 128k -- allocator without fragmentation (expandable segments), then the optimizer
# states on the host (ZeRO-Offload) to free ~96 GB of HBM for activations.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HDS_BENCH_PROGRESS=1 PYTORCH_ALLOC_CONF=expandable_segments:True
mkdir -p gpurun_out/seq
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py --micro-batch 1 "$@" > gpurun_out/seq/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/seq/summary.txt
  grep '^{' gpurun_out/seq/$name.log >> gpurun_out/seq/summary.txt
  return $rc
}
run ckpt_256k_exp 560 --seq 262144 --ckpt --steps 1 --warmup 1
run ckpt_256k_offload 560 --seq 262144 --ckpt --offload cpu --steps 1 --warmup 1
exit 0
