"""Decode-attention microbenchmark: HIP kernel (ops/decode_attention.py) vs SDPA with repeat_interleave (the old
v1 path) and SDPA with enable_gqa, over HF-layout caches. Prints one JSON line per shape (GB/s of K+V read)."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.decode_attention import decode_attention  # noqa: E402


def t(fn, it=50):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for B, H, Hkv, S, D in [(1, 32, 8, 4096, 128), (8, 32, 8, 4096, 128), (32, 32, 8, 2048, 128), (8, 32, 32, 8192, 128),
                        (16, 64, 8, 16384, 128)]:
    q = torch.randn(B, H, 1, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16)
    G = H // Hkv
    kern = t(lambda: decode_attention(q[:, :, 0], k, v, 0.088))
    rep = t(lambda: F.scaled_dot_product_attention(q, k.repeat_interleave(G, 1), v.repeat_interleave(G, 1)))
    gqa = t(lambda: F.scaled_dot_product_attention(q, k, v, enable_gqa=G > 1))
    byts = 2 * B * Hkv * S * D * 2
    print(json.dumps({"B": B, "H": H, "Hkv": Hkv, "S": S, "D": D, "hds_us": round(kern * 1e3, 1),
                      "sdpa_repeat_us": round(rep * 1e3, 1), "sdpa_gqa_us": round(gqa * 1e3, 1),
                      "hds_GBps": round(byts / kern / 1e6, 1)}), flush=True)
