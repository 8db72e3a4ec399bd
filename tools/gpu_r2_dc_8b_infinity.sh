# GPU: Llama-3-8B ZeRO-Infinity on 1 MI355X (params + optimizer in pinned host memory, CPU Adam), with / without
# DeepCompile (selective gather keeps units resident fwd->bwd: no backward H2D parameter fetches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --offload cpu --offload-param --micro-batch 2 --steps 3 --warmup 2 > gpurun_out/r2_8b_inf_base.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --offload cpu --offload-param --micro-batch 2 --steps 3 --warmup 2 --deepcompile > gpurun_out/r2_8b_inf_dc.log 2>&1 || exit 1
