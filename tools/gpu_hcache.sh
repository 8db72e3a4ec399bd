# GPU: HCache restore vs recompute vs KV-offload restore (Llama-3-8B serving engine)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true
timeout -k 10 600 python -u tools/bench_hcache.py --seqs 8 --ctx 2048 --model llama2-7b > gpurun_out/hcache_bench_l2.log 2>&1
