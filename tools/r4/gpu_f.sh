# GPU: D2H copy engine A/B for the 32k plan (runtime blit limited to 8 / 32 workgroups, own kernel at 4), headline
# with / without the blit limit, optimizer-state offload at mb10 with memory-driven per-state reload
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> gpurun_out/r4f/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230 --act-cache-policy plan --act-cache-spill-overlap 0.8"
HDS_D2H_WG=0 DEBUG_CLR_LIMIT_BLIT_WG=8 run timeout -k 10 300 $B > gpurun_out/r4f/plan_blit8.log 2>&1
HDS_D2H_WG=0 DEBUG_CLR_LIMIT_BLIT_WG=32 run timeout -k 10 300 $B > gpurun_out/r4f/plan_blit32.log 2>&1
HDS_D2H_WG=4 run timeout -k 10 300 $B > gpurun_out/r4f/plan_wg4.log 2>&1
HDS_D2H_WG=0 DEBUG_CLR_LIMIT_BLIT_WG=16 run timeout -k 10 300 $B > gpurun_out/r4f/plan_blit16.log 2>&1
run timeout -k 10 300 python -u bench.py --seq 32768 --micro-batch 1 --steps 4 --warmup 5 --host-act-cache --act-cache-budget-gib 230 --act-cache-policy recompute > gpurun_out/r4f/recompute.log 2>&1
run timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4f/bench_default.log 2>&1
DEBUG_CLR_LIMIT_BLIT_WG=16 run timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4f/bench_blit16.log 2>&1
run timeout -k 10 300 python -u bench.py --micro-batch 10 --steps 4 --warmup 3 --offload-opt-states > gpurun_out/r4f/mb10_offstates100.log 2>&1
