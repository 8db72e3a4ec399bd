# GPU: NVMe tier test + 70B-width NVMe bench (reduced layers, valid:false) + 32k long-context comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
df -h /tmp > gpurun_out/r2_df.txt 2>&1
free -g >> gpurun_out/r2_df.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_host_tier_gpu.py > gpurun_out/r2_nvme_test.log 2>&1 || { echo "rc=$?" >> gpurun_out/r2_nvme_test.log; exit 1; }
timeout -k 10 900 python -u bench.py --model llama3-70b --layers 2 --offload nvme --offload-param --micro-batch 1 --seq 4096 --steps 2 --warmup 1 > gpurun_out/r2_bench70b_nvme.log 2>&1 || { echo "rc=$?" >> gpurun_out/r2_bench70b_nvme.log; exit 1; }
rm -rf /tmp/hds_nvme
timeout -k 10 600 python -u bench.py --seq 32768 --micro-batch 1 --ckpt --steps 3 --warmup 1 > gpurun_out/r2_bench32k_ckpt.log 2>&1 || echo "rc=$?" >> gpurun_out/r2_bench32k_ckpt.log
timeout -k 10 600 python -u bench.py --seq 32768 --micro-batch 1 --host-act-cache --steps 3 --warmup 1 > gpurun_out/r2_bench32k_actcache.log 2>&1 || echo "rc=$?" >> gpurun_out/r2_bench32k_actcache.log
