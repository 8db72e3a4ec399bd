"""Does weight-pointer alignment (flat-buffer views) change hipBLASLt GEMM speed? + sustained-run clocks."""
import time
import torch

T = 16384


def bench(fn, flops, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / it
    return flops / dt / 1e12


for name, (K, N) in {"gate_up": (4096, 28672), "down": (14336, 4096), "o": (4096, 4096)}.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    f = 2 * T * N * K
    row = []
    for off in (0, 8, 64, 128):
        buf = torch.randn(N * K + 256, device="cuda", dtype=torch.bfloat16)
        W = buf[off:off + N * K].view(N, K)
        row.append(f"off{off}: fwd {bench(lambda: x @ W.t(), f):.0f} dgrad {bench(lambda: dy @ W, f):.0f} "
                   f"wgrad {bench(lambda: dy.t() @ x, f):.0f}")
    print(name, " | ".join(row), flush=True)

# sustained: 30 s of back-to-back gate_up fwd GEMMs, report TF per 2 s window
K, N = 4096, 28672
x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
f = 2 * T * N * K
t0 = time.time()
while time.time() - t0 < 30:
    print(f"t={time.time() - t0:5.1f}s sustained fwd {bench(lambda: x @ W.t(), f, it=200):.0f} TF", flush=True)
