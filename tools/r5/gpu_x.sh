# GPU: plan policy under the default budget after the first-plan margin: 32k x mb2 and 64k x mb1 (all-step peaks),
# and the budget-cap GPU test
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5x
mkdir -p $O
export HDS_BENCH_PROGRESS=1
timeout -k 10 420 python -u bench.py --seq 32768 --micro-batch 2 --steps 4 --warmup 6 --host-act-cache --act-cache-policy plan --act-cache-spill-overlap 0.8 > $O/plan_32768_mb2.log 2>&1
echo "plan32k rc=$?" >> $O/status.txt
timeout -k 10 420 python -u bench.py --seq 65536 --micro-batch 1 --steps 4 --warmup 6 --host-act-cache --act-cache-policy plan --act-cache-spill-overlap 0.8 > $O/plan_65536_mb1.log 2>&1
echo "plan64k rc=$?" >> $O/status.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_act_plan_gpu.py -k budget_is_a_cap > $O/budget_cap.log 2>&1
echo "cap rc=$?" >> $O/status.txt
exit 0
