"""Does a pinned D2H / H2D copy on a side stream overlap GEMMs on the compute stream? (wall times)"""
import sys
import time

sys.path.insert(0, ".")

import torch

dev = torch.device("cuda")
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
src = torch.randn((1 << 30) // 2, device=dev, dtype=torch.bfloat16)  # 1 GiB
host = torch.empty(src.numel(), dtype=src.dtype, pin_memory=True)
side = torch.cuda.Stream()


def gemms(n=60):
    for _ in range(n):
        torch.matmul(a, b)


def t(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


for _ in range(2):
    gemms(5)
    host.copy_(src, non_blocking=True)
tg = t(gemms)
td = t(lambda: host.copy_(src, non_blocking=True))
th = t(lambda: src.copy_(host, non_blocking=True))


def both(d2h=True):
    with torch.cuda.stream(side):
        for _ in range(4):
            (host.copy_(src, non_blocking=True) if d2h else src.copy_(host, non_blocking=True))
    gemms()


tb = t(both)
tb2 = t(lambda: both(False))
print(f"gemms {tg:.1f} ms | D2H 1GiB {td:.1f} ms ({1/td*1e3:.1f} GiB/s) | H2D 1GiB {th:.1f} ms | "
      f"gemms + 4xD2H on side stream {tb:.1f} ms (serial would be {tg + 4*td:.1f}) | "
      f"gemms + 4xH2D {tb2:.1f} ms (serial {tg + 4*th:.1f})")

# same, with this framework's pinned pool buffers (offload/pinned.py) and the cache's event pattern
from hcache_deepspeed_amd.offload.pinned import PinnedPool  # noqa: E402

pool = PinnedPool()
hbuf = pool.get(src.numel(), src.dtype)
print("pool buffer is_pinned:", hbuf.is_pinned())


def both_pool():
    cur = torch.cuda.current_stream()
    for _ in range(4):
        dst = torch.empty_like(src)
        ready = torch.cuda.Event()
        ready.record(cur)
        with torch.cuda.stream(side):
            side.wait_event(ready)
            dst.copy_(hbuf, non_blocking=True)
            dst.record_stream(side)
    gemms()


tp = t(both_pool)
print(f"gemms + 4xH2D from pool buffers with ready events: {tp:.1f} ms (serial {tg + 4*th:.1f})")
