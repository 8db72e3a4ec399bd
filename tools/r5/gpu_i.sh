# GPU: budget-cap test after the in-budget copy window; then the default-budget shapes (gpu_e)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_act_plan_gpu.py -k budget_is_a_cap -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "rc=$rc tests" >> $O/status.txt
case $rc in 124|134|137|139) exit $rc;; esac
bash tools/r5/gpu_e.sh
exit 0
