"""When does the HIP runtime read DEBUG_CLR_LIMIT_BLIT_WG? GEMMs on the compute stream beside 4 x 1 GiB pinned D2H
copies on a side stream, with the limit set (a) in the environment before the process starts (run with it exported),
(b) from Python after `import torch` but before the first device call (argv[1] == "late"), (c) not at all.
The GEMM slowdown from the copies' blit kernels tells which settings took effect."""
import os
import sys
import time

import torch

if len(sys.argv) > 1 and sys.argv[1] == "late":
    os.environ["DEBUG_CLR_LIMIT_BLIT_WG"] = "16"
dev = torch.device("cuda")
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
src = torch.randn((1 << 30) // 2, device=dev, dtype=torch.bfloat16)
host = torch.empty(src.numel(), dtype=src.dtype, pin_memory=True)
side = torch.cuda.Stream()


def gemms(n=200):  # ~0.2 s: longer than the 4 GiB of copies, so the wall time is the GEMMs
    for _ in range(n):
        torch.matmul(a, b)


def t(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def both():
    with torch.cuda.stream(side):
        for _ in range(4):
            host.copy_(src, non_blocking=True)
    gemms()


for _ in range(2):
    gemms(5)
    both()
tg = min(t(gemms) for _ in range(3))
tb = min(t(both) for _ in range(3))
print(f"mode={sys.argv[1] if len(sys.argv) > 1 else 'env:' + os.environ.get('DEBUG_CLR_LIMIT_BLIT_WG', 'unset')} "
      f"gemms {tg:.1f} ms, gemms + 4 GiB D2H beside {tb:.1f} ms (+{100 * (tb / tg - 1):.1f} %)", flush=True)
