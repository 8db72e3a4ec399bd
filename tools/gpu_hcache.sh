# GPU: HCache restore vs recompute vs KV-offload restore (Llama-3-8B serving engine)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inference_v2.py tests/test_inference_v2_families.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/hcache_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_hcache.py --seqs 8 --ctx 2048 > gpurun_out/hcache_bench.log 2>&1
