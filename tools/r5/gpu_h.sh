# GPU: budget-cap + graph-decode fp8 latent tests; 128k / 320k ckpt_offload with the summed boundary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
run() {
  "$@"; rc=$?
  echo "rc=$rc: $*" >> $O/status.txt
  case $rc in 124|134|137|139) exit $rc;; esac
  return $rc
}
run timeout -k 10 400 python -u -m pytest tests/test_act_plan_gpu.py -k budget_is_a_cap tests/test_inference_v2.py -k "budget_is_a_cap or graph_decode_captures" -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1
bash tools/r5/gpu_g.sh
exit 0
