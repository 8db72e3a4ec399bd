"""Decode-time weight-only INT8/INT4 GEMV vs the bf16 hipBLASLt GEMM (Llama-3-8B projection shapes, M = 1..8)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hcache_deepspeed_amd.ops import quantizer as Q  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    dev = torch.device("cuda", 0)
    for N, K in ((6144, 4096), (28672, 4096), (4096, 14336), (128256, 4096)):
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        for bits in (8, 4):
            q, s, _ = Q.quantize(w.reshape(-1).contiguous(), 128, bits, True)
            for M in (1, 2, 8):
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                tq = timeit(lambda: Q.int_linear(x, q, s, N, K, 128, bits))
                tb = timeit(lambda: torch.nn.functional.linear(x, w))
                gbs = (q.numel() + s.numel() * 4) / tq / 1e9
                print(f"N={N:6d} K={K:5d} M={M} int{bits}: {tq*1e6:8.1f} us ({gbs:6.0f} GB/s weight stream) | "
                      f"bf16 hipBLASLt {tb*1e6:8.1f} us | speedup {tb/tq:4.2f}x", flush=True)


if __name__ == "__main__":
    main()
