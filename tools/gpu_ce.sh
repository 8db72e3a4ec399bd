# GPU: kernel tests (incl. fused linear CE grads) + default bench after folding the LM-head grad accumulation
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_kernels_ce.log 2>&1 || exit 1
timeout -k 10 200 python -c "import torch; from hcache_deepspeed_amd.ops import cross_entropy as C; a=torch.zeros(64,32,device='cuda'); x=torch.randn(64,16,device='cuda',dtype=torch.bfloat16); y=torch.randn(16,32,device='cuda',dtype=torch.bfloat16); C._addmm_f32_(a,x,y); C._addmm_f32_(a,x,y); r=2*(x.float()@y.float()); print('fused', C._ADDMM_OUT_DTYPE[0], 'err', (a-r).abs().max().item())" > gpurun_out/addmm_check.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_ce.log 2>&1
