# GPU: qkv split forward, the headline bench + kernel stats, the copy/fill op census, the NVMe ceiling; last: the
# down-projection split-K wgrad diagnosis, each layout in its own short-lived process
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rc
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
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_symmetric_gpu.py > gpurun_out/rc/symm.log 2>&1 || exit 1
for lay in direct nt direct_sk2 nt_sk2; do
  timeout -k 5 60 python -u tools/r3/wgrad_down_diag.py $lay >> gpurun_out/rc/down_diag.log 2>&1 || exit 1
done
