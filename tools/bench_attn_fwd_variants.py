"""Sweep the FlashAttention forward variants (static priority / deferred max) at the bench shape
(Llama-3-8B heads, B=7, S=4096, causal) and report TF/s plus the max deviation from variant 0 and from an fp32
reference on a slice."""
import sys
import time

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops import native  # noqa: E402
from hcache_deepspeed_amd.ops.attention import flash_attn  # noqa: E402


def timeit(fn, iters=20):
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
    fl = 4 * B * Hq * S * S * D / 2
    lib = native.kernels()
    # fp32 reference for batch 0, heads 0..3
    qf, kf, vf = q[0, :, :4].float().transpose(0, 1), k[0, :, :1].float().transpose(0, 1), v[0, :, :1].float().transpose(0, 1)
    s = (qf @ kf.transpose(-1, -2)) / D**0.5
    s = s.masked_fill(torch.triu(torch.ones(S, S, device="cuda", dtype=torch.bool), 1), float("-inf"))
    ref = (torch.softmax(s, -1) @ vf).transpose(0, 1)
    base = None
    vs = [int(x) for x in sys.argv[1].split(',')] if len(sys.argv) > 1 else [2, 4, 5, 2, 5]
    for var in vs:
        lib.hds_attn_fwd_variant(var)
        o = flash_attn(q, k, v, causal=True)
        t = timeit(lambda: flash_attn(q, k, v, causal=True))
        if base is None:
            base = o.clone()
        d0 = (o.float() - base.float()).abs().max().item()
        dr = (o[0, :, :4].float() - ref).abs().max().item()
        print(f"fwd variant {var}: {t*1e3:.3f} ms {fl/t/1e12:.0f} TF/s | max|o-o_v0| {d0:.3e} | max|o-ref32| {dr:.3e}",
              flush=True)
    lib.hds_attn_fwd_variant(2)
    do = torch.randn_like(q)
    qg, kg, vg = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    grads0 = None
    for prio in (() if len(sys.argv) > 2 else (1,)):
        lib.hds_attn_bwd_prio(prio)

        def fb():
            qg.grad = kg.grad = vg.grad = None
            flash_attn(qg, kg, vg, causal=True).backward(do)

        tfb = timeit(fb, 10)
        tf = timeit(lambda: flash_attn(qg, kg, vg, causal=True), 10)
        fb()
        g = (qg.grad.clone(), kg.grad.clone(), vg.grad.clone())
        grads0 = grads0 or g
        d = max((a.float() - b.float()).abs().max().item() for a, b in zip(g, grads0))
        print(f"bwd prio {prio}: {(tfb-tf)*1e3:.3f} ms {2.5*fl/(tfb-tf)/1e12:.0f} TF/s | maxdiff vs prio0 {d:.3e}",
              flush=True)
    lib.hds_attn_bwd_prio(0)


if __name__ == "__main__":
    main()
