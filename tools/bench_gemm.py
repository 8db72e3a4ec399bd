"""Per-shape GEMM throughput for the Llama-3-8B layer GEMMs (fwd / dgrad / wgrad) in every layout."""
import torch
import time

T = 24576
shapes = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
          "lm_head_chunk": (4096, 128256)}


def bench(fn, flops, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / it
    return flops / dt / 1e12, dt * 1e3


dev = "cuda"
for name, (K, N) in shapes.items():
    M = 4096 if name == "lm_head_chunk" else T
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    W = torch.randn(N, K, device=dev, dtype=torch.bfloat16)  # nn.Linear layout [out, in]
    Wt = W.t().contiguous()                                   # [in, out]
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    f = 2 * M * N * K
    r = {}
    r["fwd x@W.T"] = bench(lambda: x @ W.t(), f)
    r["fwd x@Wt"] = bench(lambda: x @ Wt, f)
    r["dgrad dy@W"] = bench(lambda: dy @ W, f)
    r["dgrad dy@Wt.T"] = bench(lambda: dy @ Wt.t(), f)
    r["wgrad dy.T@x"] = bench(lambda: dy.t() @ x, f)
    r["wgrad x.T@dy"] = bench(lambda: x.t() @ dy, f)
    print(name, M, K, N, " | ".join(f"{k}: {v[0]:.0f} TF ({v[1]:.2f} ms)" for k, v in r.items()), flush=True)
