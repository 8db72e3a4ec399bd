# GPU: headline bench with and without the NT-layout input-gradient GEMMs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_nt1.log 2>&1 || exit 1
HDS_NT_DGRAD=0 timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_nt0.log 2>&1
