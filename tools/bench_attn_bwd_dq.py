"""Time the FlashAttention backward at the bench shape (Llama-3-8B heads, B=7, S=4096, causal) with each dQ kernel
variant (hds_attn_bwd_dq_variant: 0 = 8 waves x 32 rows, 1 = one wave per SIMD x 64 rows) and report the backward
in ms / nominal TF/s (2.5x the forward's FLOPs) plus the dQ deviation from variant 0."""
import sys
import time

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops import native  # noqa: E402
from hcache_deepspeed_amd.ops.attention import flash_attn  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    B, S, Hq, Hkv, D = 7, 4096, 32, 8, 128
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    do = torch.randn_like(q)
    fl = 4 * B * Hq * S * S * D / 2
    lib = native.kernels()
    qg, kg, vg = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    base = None
    vs = [int(x) for x in sys.argv[1].split(',')] if len(sys.argv) > 1 else [0, 1, 0, 1]
    for var in vs:
        lib.hds_attn_bwd_dq_variant(var)

        def fb():
            qg.grad = kg.grad = vg.grad = None
            flash_attn(qg, kg, vg, causal=True).backward(do)

        tfb = timeit(fb)
        tf = timeit(lambda: flash_attn(qg, kg, vg, causal=True))
        fb()
        dq = qg.grad.float().clone()
        base = dq if base is None else base
        rel = ((dq - base).norm() / base.norm()).item()
        print(f"dq variant {var}: bwd {(tfb - tf) * 1e3:.3f} ms {2.5 * fl / (tfb - tf) / 1e12:.0f} TF/s | "
              f"fwd {tf * 1e3:.3f} ms | rel dq vs first {rel:.2e}", flush=True)
    lib.hds_attn_bwd_dq_variant(0)


if __name__ == "__main__":
    main()
