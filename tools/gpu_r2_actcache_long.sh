set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HDS_BENCH_PROGRESS=1
mkdir -p gpurun_out/seq
run() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py --micro-batch 1 "$@" > gpurun_out/seq/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/seq/summary_cache.txt
  grep '^{' gpurun_out/seq/$name.log >> gpurun_out/seq/summary_cache.txt
  return $rc
}
run cache_64k 400 --seq 65536 --host-act-cache --steps 2 --warmup 2
run cache_128k_offload 700 --seq 131072 --host-act-cache --offload cpu --steps 1 --warmup 2
exit 0
