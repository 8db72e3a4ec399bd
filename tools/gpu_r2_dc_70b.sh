# GPU: ZeRO-Infinity Llama-3-70B width (2 layers, params + optimizer on the NVMe tier), with / without DeepCompile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --model llama3-70b --layers 2 --offload nvme --offload-param --micro-batch 1 --seq 4096 --steps 3 --warmup 2 > gpurun_out/r2_70b_nvme_base.log 2>&1 || exit 1
rm -rf /tmp/hds_nvme
timeout -k 10 600 python -u bench.py --model llama3-70b --layers 2 --offload nvme --offload-param --micro-batch 1 --seq 4096 --steps 3 --warmup 2 --deepcompile > gpurun_out/r2_70b_nvme_dc.log 2>&1 || exit 1
rm -rf /tmp/hds_nvme
