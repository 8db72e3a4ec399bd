"""Decode-sized bf16 linear: HIP GEMV (ops/gemv.py) against F.linear (hipBLASLt) at Llama-3-8B projection shapes,
M = 1, 4, 8 rows; also checks the result against an fp32 reference."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.gemv import gemv  # noqa: E402


def t(fn, it=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
                       ("lm_head", 128256, 4096)):
        w = (torch.randn(N, K, device="cuda", generator=g) * K**-0.5).to(torch.bfloat16)
        for M in (1, 4, 8):
            x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
            y = gemv(x, w)
            ref = x.float() @ w.float().t()
            rel = ((y.float() - ref).norm() / ref.norm()).item()
            tg, tl = t(lambda: gemv(x, w)), t(lambda: F.linear(x, w))
            print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "gemv_us": round(tg, 2), "hipblaslt_us": round(tl, 2),
                              "gemv_TBps": round(N * K * 2 / tg / 1e6, 2), "speedup": round(tl / tg, 3),
                              "rel_err": rel}), flush=True)


if __name__ == "__main__":
    main()
