# GPU: rocprofv3 timeline of the 32k activation plan (kernel + memory-copy trace, last step), optimizer-state offload
# at mb10 with every state offloaded
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4d/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4d/plan32k -o run -- python3 bench.py --seq 32768 --micro-batch 1 --host-act-cache --act-cache-policy plan --act-cache-budget-gib 230 --act-cache-spill-overlap 0.8 --steps 1 --warmup 5 > gpurun_out/r4d/plan32k.log 2>&1
run python3 tools/r4/step_timeline.py gpurun_out/r4d/plan32k > gpurun_out/r4d/plan32k_timeline.txt 2>&1
find gpurun_out/r4d -name "*.csv" -size +40M -delete
run timeout -k 10 300 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states > gpurun_out/r4d/mb10_offstates100.log 2>&1
