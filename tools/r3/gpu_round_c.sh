# GPU: FA backward pipelining (tests + A/B), split-K wgrad micro-benchmark + layout tests, qkv split forward, then
# the headline bench + kernel stats, the copy/fill op census and the NVMe ceiling
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rc
ok_or_fail() { if [ $1 -ne 0 ] && [ $1 -ne 1 ]; then echo "fatal rc=$1"; exit $1; fi; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/rc/flash_tests.log 2>&1
rc=$?; echo "flash tests rc=$rc"; ok_or_fail $rc
if [ $rc -ne 0 ]; then export HDS_ATTN_BWD_PIPE=0; fi
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad_layout_gpu.py > gpurun_out/rc/wgrad_tests.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; ok_or_fail $rc
if [ $rc -ne 0 ]; then export HDS_WGRAD_LAYOUT=direct; fi
HDS_ATTN_BWD_PIPE=0 timeout -k 10 120 python -u tools/r3/fa_bench.py > gpurun_out/rc/fa_pipe0.log 2>&1 || exit 1
HDS_ATTN_BWD_PIPE=1 timeout -k 10 120 python -u tools/r3/fa_bench.py > gpurun_out/rc/fa_pipe1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_wgrad_layout.py --splitk > gpurun_out/rc/wgrad_splitk.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_qkv_split.py --slices > gpurun_out/rc/qkv_slices.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rc/bench.log 2>&1 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rc/prof -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/rc/prof.log 2>&1 || exit 1
find gpurun_out/rc -name "*kernel_trace.csv" -delete
timeout -k 10 300 python -u tools/r3/aten_op_census.py > gpurun_out/rc/census.log 2>&1 || exit 1
df -h /tmp > gpurun_out/rc/ds_io.log 2>&1
for qd in 32 128; do
  timeout -k 10 120 python -u -m hcache_deepspeed_amd.nvme.ds_io --folder /tmp/hds_nvme --io_size 8G --write --queue_depth $qd --threads 8 --block_size 4M >> gpurun_out/rc/ds_io.log 2>&1 || exit 1
  timeout -k 10 120 python -u -m hcache_deepspeed_amd.nvme.ds_io --folder /tmp/hds_nvme --io_size 8G --read --queue_depth $qd --threads 8 --block_size 4M >> gpurun_out/rc/ds_io.log 2>&1 || exit 1
done
rm -rf /tmp/hds_nvme
