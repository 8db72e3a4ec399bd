"""Mixed-input MFMA GEMM vs bf16 hipBLASLt at Llama-3-8B projection shapes (1 x MI355X)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops import quantizer as Q  # noqa: E402


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for name, (N, K) in shapes.items():
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        q8, s8, _ = Q.quantize(w.reshape(-1), 128, 8, True)
        q4, s4, _ = Q.quantize(w.reshape(-1), 128, 4, True)
        q6, s6 = Q.quantize_minifloat(w.reshape(-1), 128, 6, 2)
        for M in (16, 32, 64, 128, 256):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            tb = t(lambda: torch.nn.functional.linear(x, w))
            t8 = t(lambda: Q.wmix_gemm(x, q8, s8, N, K, 128, "int8"))
            t4 = t(lambda: Q.wmix_gemm(x, q4, s4, N, K, 128, "int4"))
            t6 = t(lambda: Q.wmix_gemm(x, q6, s6, N, K, 128, "fp6", 3))
            td = t(lambda: torch.nn.functional.linear(x, Q.dequantize(q8, s8, None, 128, 8, True).view(N, K)))
            print(f"{name:8s} N={N:6d} K={K:6d} M={M:4d} | bf16 {tb*1e6:7.1f} us ({N*K*2/tb/1e12:4.2f} TB/s) | "
                  f"int8 {t8*1e6:7.1f} us ({tb/t8:4.2f}x, {N*K/t8/1e12:4.2f} TB/s) | int4 {t4*1e6:7.1f} us "
                  f"({tb/t4:4.2f}x) | fp6 {t6*1e6:7.1f} us ({tb/t6:4.2f}x) | int8 dequant+gemm {td*1e6:7.1f} us",
                  flush=True)


if __name__ == "__main__":
    main()
