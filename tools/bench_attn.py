"""Micro-benchmark of the HIP FlashAttention kernels (Llama-3-8B shapes) against torch SDPA."""
import math
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
    B, S, Hq, Hkv, D = 2, 4096, 32, 8, 128
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    fl_fwd = 4 * B * Hq * S * S * D / 2
    lib = native.kernels()
    ref = None
    for cfg in [(4, 4, 4), (8, 4, 8), (8, 8, 8)]:
        lib.hds_attn_config(*cfg)
        o = flash_attn(q, k, v, causal=True)
        tf = timeit(lambda: flash_attn(q, k, v, causal=True))
        def fb():
            q.grad = k.grad = v.grad = None
            flash_attn(q, k, v, causal=True).backward(do)
        tfb = timeit(fb)
        fb()
        grads = (q.grad.clone(), k.grad.clone(), v.grad.clone())
        if ref is None:
            ref = (o.detach().clone(), grads)
        err = max((a.float() - b.float()).abs().max().item() for a, b in zip((o, ) + grads, (ref[0], ) + ref[1]))
        tb = tfb - tf
        print(f"cfg fwd/dkdv/dq waves={cfg}: fwd {tf*1e3:.3f} ms {fl_fwd/tf/1e12:.0f} TF/s | bwd {tb*1e3:.3f} ms "
              f"{2.5*fl_fwd/tb/1e12:.0f} TF/s | maxdiff vs first {err:.3e}", flush=True)
    lib.hds_attn_config(8, 4, 8)
    # torch SDPA (ROCm flash backend) on the same shapes for reference
    try:
        qt, kt, vt = (t.detach().transpose(1, 2).contiguous().requires_grad_(True) for t in (q, k, v))
        kt2 = kt.detach().repeat_interleave(Hq // Hkv, 1).requires_grad_(True)
        vt2 = vt.detach().repeat_interleave(Hq // Hkv, 1).requires_grad_(True)
        f = lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt2, vt2, is_causal=True)
        tf = timeit(f)
        dot = do.transpose(1, 2).contiguous()
        def fb2():
            qt.grad = kt2.grad = vt2.grad = None
            f().backward(dot)
        tfb = timeit(fb2)
        print(f"torch SDPA: fwd {tf*1e3:.3f} ms {fl_fwd/tf/1e12:.0f} TF/s | bwd {(tfb-tf)*1e3:.3f} ms "
              f"{2.5*fl_fwd/(tfb-tf)/1e12:.0f} TF/s")
    except Exception as e:  # pragma: no cover
        print("torch SDPA unavailable:", e)


if __name__ == "__main__":
    main()
