# GPU: chunked optimizer-state offload test on the device
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_host_tier_gpu.py -k "chunked_state_offload" > $O/test.log 2>&1
echo "rc=$?" >> $O/status.txt
tail -5 $O/test.log
