"""Evoformer attention forward: HIP kernel vs the chunked-GEMM path (AlphaFold MSA row attention shapes)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hcache_deepspeed_amd.ops.deepspeed4science.evoformer_attn as ev  # noqa: E402


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it


dev = torch.device("cuda", 0)
for (B, N, L, H, D) in ((1, 256, 256, 8, 32), (1, 128, 512, 8, 32), (1, 64, 768, 4, 64)):
    q, k, v = (torch.randn(B, N, L, H, D, device=dev, dtype=torch.bfloat16) for _ in range(3))
    b1 = torch.zeros(B, N, 1, 1, L, device=dev, dtype=torch.bfloat16)
    b2 = torch.randn(B, 1, H, L, L, device=dev, dtype=torch.bfloat16)
    flops = 4.0 * B * N * H * L * L * D
    with torch.no_grad():
        th = timeit(lambda: ev.DS4Sci_EvoformerAttention(q, k, v, [b1, b2]))
        orig = ev._hip_eligible
        ev._hip_eligible = lambda *a: False
        tc = timeit(lambda: ev.DS4Sci_EvoformerAttention(q, k, v, [b1, b2]))
        ev._hip_eligible = orig
    print(f"B={B} N={N} L={L} H={H} D={D}: HIP {th*1e3:7.2f} ms ({flops/th/1e12:6.1f} TF/s) | chunked GEMM path "
          f"{tc*1e3:7.2f} ms | speedup {tc/th:4.2f}x", flush=True)
