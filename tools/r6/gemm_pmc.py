"""hipBLASLt at the headline's GEMM shapes, for a rocprofv3 PMC pass (clock and MFMA busy): each shape runs 10 times
on random N(0,1) bf16 operands (zeros would read high: DVFS). Prints wall TFLOP/s per shape (events)."""
import json
import sys

import torch

SHAPES = [(28672, 28672, 4096, "gate_up fwd NT"), (28672, 4096, 14336, "down fwd NT"),
          (28672, 6144, 4096, "qkv fwd NT"), (28672, 4096, 4096, "o fwd NT")]
for M, N, K, name in SHAPES:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, b.t(), out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.matmul(a, b.t(), out=c)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "ms": round(ms, 3),
                      "tflops": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)
    del a, b, c
    torch.cuda.empty_cache()
