# GPU: host-tier and FlashAttention GPU tests on the final tree
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ba
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_host_tier_gpu.py tests/test_kernels_gpu.py -k "host_tier or twin or host_step or state_offload or flash" > $O/test.log 2>&1
echo "rc=$?" >> $O/status.txt
tail -2 $O/test.log
