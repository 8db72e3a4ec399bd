"""Grouped MoE GEMM micro-benchmark on MI355X: HIP grouped kernel vs hipBLASLt per-expert GEMMs (which need
the routing counts on the host), at Mixtral-8x7B expert shapes (H=4096, I=14336, 8 experts, top-2) for several token counts."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hcache_deepspeed_amd.ops.grouped_gemm import expert_offsets, grouped_gemm


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    dev = torch.device("cuda", 0)
    E, H, I = 8, 4096, 14336
    quick = "--quick" in sys.argv
    for T in ((8192, ) if quick else (256, 2048, 8192, 32768)):
        torch.manual_seed(0)
        rows = T * 2
        counts = torch.distributions.Multinomial(rows, torch.ones(E)).sample().long()
        offs = expert_offsets(counts.to(dev))
        x = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
        for name, N, K in (("w13", 2 * I, H), ("w2", H, I)):
            w = torch.randn(E, N, K, device=dev, dtype=torch.bfloat16) / K**0.5
            xi = x if K == H else torch.randn(rows, K, device=dev, dtype=torch.bfloat16)
            flops = 2.0 * rows * N * K
            o = counts.tolist()
            starts = [0]
            for c in o:
                starts.append(starts[-1] + c)
            t_g1 = timeit(lambda: grouped_gemm(xi, w, offs, variant=1))
            t_g = timeit(lambda: grouped_gemm(xi, w, offs, variant=2))
            t_l = timeit(lambda: [xi[starts[e]:starts[e + 1]] @ w[e].t() for e in range(E)])
            ref = torch.cat([xi[starts[e]:starts[e + 1]].float() @ w[e].float().t() for e in range(E)])
            err = max((grouped_gemm(xi, w, offs, variant=v).float() - ref).abs().max().item() for v in (1, 2))
            print(f"T={T:6d} {name} rows={rows:6d} N={N:5d} K={K:5d} | grouped128 {t_g1*1e3:7.3f} ms "
                  f"{flops/t_g1/1e12:6.1f} TF/s | grouped256 {t_g*1e3:7.3f} ms {flops/t_g/1e12:6.1f} TF/s | per-expert hipBLASLt {t_l*1e3:7.3f} ms {flops/t_l/1e12:6.1f} TF/s | "
                  f"max err {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
