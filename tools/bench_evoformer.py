"""Evoformer attention fwd+bwd timing: HIP kernels vs the chunked torch path, MSA-row-attention shapes."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.deepspeed4science import evoformer_attn as ev  # noqa: E402


def run(B, N, L, H, D, hip):
    q, k, v = (torch.randn(B, N, L, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    b1 = torch.zeros(B, N, 1, 1, L, device="cuda", dtype=torch.bfloat16)
    b2 = torch.randn(B, 1, H, L, L, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    orig = ev._hip_eligible
    if not hip:
        ev._hip_eligible = lambda *a: False
    try:
        for _ in range(2):
            ev.DS4Sci_EvoformerAttention(q, k, v, [b1, b2]).sum().backward()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            ev.DS4Sci_EvoformerAttention(q, k, v, [b1, b2]).sum().backward()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / 5 * 1e3
    finally:
        ev._hip_eligible = orig


for shape in [(1, 128, 256, 8, 32), (1, 64, 512, 8, 32), (1, 256, 384, 4, 64)]:
    print(json.dumps({"B,N,L,H,D": shape, "hip_fwd_bwd_ms": round(run(*shape, True), 2),
                      "torch_chunked_fwd_bwd_ms": round(run(*shape, False), 2)}), flush=True)
