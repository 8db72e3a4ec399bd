# GPU: v2 decode time split (graph vs eager) and the 32k host activation cache after the copy-window change
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rd
timeout -k 10 300 python -u tools/r3/v2_decode_diag.py > gpurun_out/rd/v2_diag.jsonl 2> gpurun_out/rd/v2_diag.err || exit 1
B="python -u bench.py --seq 32768 --micro-batch 1 --steps 3 --warmup 2"
timeout -k 10 400 $B --host-act-cache --act-cache-budget-gib 230 > gpurun_out/rd/ac32k_b230.log 2>&1 || exit 1
timeout -k 10 400 $B --host-act-cache > gpurun_out/rd/ac32k.log 2>&1 || exit 1
timeout -k 10 400 $B --ckpt > gpurun_out/rd/ckpt32k.log 2>&1 || exit 1
# DeepCompile offload_parameters at dp1 (every shard on the host / pass keeps 8 GiB on the device)
timeout -k 10 400 python -u bench.py --steps 5 --warmup 3 --offload-params-compile 0 > gpurun_out/rd/offp_0.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 3 --offload-params-compile 8 > gpurun_out/rd/offp_8.log 2>&1 || exit 1
