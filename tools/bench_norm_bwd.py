"""RMSNorm backward (fused residual-gradient add) at the bench shape [28672, 4096] bf16: time and effective HBM
rate against the workgroup cap (= fp32 weight-gradient partial rows)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops import native  # noqa: E402
from hcache_deepspeed_amd.ops.norm import _native_bwd  # noqa: E402


def main():
    rows, cols = 28672, 4096
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn(rows, cols, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(rows, cols, device="cuda", generator=g).to(torch.bfloat16)
    dres = torch.randn(rows, cols, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randn(cols, device="cuda", generator=g).to(torch.bfloat16)
    rstd = torch.rsqrt(h.float().pow(2).mean(-1) + 1e-6)
    lib = native.kernels()
    ref = None
    for cap in (512, 1024, 2048, 4096):
        lib.hds_norm_bwd_set_max_parts(cap)
        fn = lambda: _native_bwd(dy, h, dres, w, None, None, rstd, False, True)  # noqa: E731
        out = fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 20
        if ref is None:
            ref = out
        err = max((a.float() - b.float()).abs().max().item() for a, b in zip(out[:2], ref[:2]))
        print(json.dumps({"cap": cap, "ms": round(ms, 4), "GBps": round(4 * rows * cols * 2 / ms / 1e6, 1),
                          "max_diff_vs_512": err}), flush=True)
    lib.hds_norm_bwd_set_max_parts(512)


if __name__ == "__main__":
    main()
