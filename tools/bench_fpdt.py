"""FPDT attention (parallel/fpdt.py: chunked causal attention, every chunk's q / k / v / o / lse parked in pinned host
memory between forward and backward, prefetched back chunk by chunk) against the plain fused-QKV attention on one
MI355X at Llama-3-8B attention width (H 4096, 32 / 8 heads, D 128): time of one forward + backward of the layer
core (qkv projection, RoPE, attention), the HBM it holds between forward and backward (what a training step keeps
per layer) and its transient peak. One JSON line per config.

Usage: python tools/bench_fpdt.py [S,...] [chunks]"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.attention import qkv_attention  # noqa: E402
from hcache_deepspeed_amd.ops.rope import rope_tables  # noqa: E402
from hcache_deepspeed_amd.parallel.fpdt import fpdt_attention  # noqa: E402

H, NQ, NKV, D = 4096, 32, 8, 128


def plain(x, w, cos, sin, S):
    T = x.shape[0]
    qkv = torch.nn.functional.linear(x, w).view(T, NQ + 2 * NKV, D)
    return qkv_attention(qkv, NQ, NKV, cos, sin, seq_len=S, causal=True).reshape(T, -1)


def run(kind, S, chunks):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = (torch.randn(S, H, device=dev) * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn((NQ + 2 * NKV) * D, H, device=dev) * 0.02).bfloat16().requires_grad_(True)
    cos, sin = rope_tables(S, D, device=dev)
    g = torch.randn(S, NQ * D, device=dev, dtype=torch.bfloat16)

    held = [0]

    def step():
        a0 = torch.cuda.memory_allocated()
        if kind == "plain":
            y = plain(x, w, cos, sin, S)
        else:
            y = fpdt_attention(x, w, None, cos, sin, NQ, NKV, D, None, 1, chunks, offload=True)
        held[0] = torch.cuda.memory_allocated() - a0 - y.numel() * y.element_size()  # saved for backward
        torch.autograd.grad(y, (x, w), g)

    step()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    t0 = time.perf_counter()
    n = 2
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    flops = 4 * NQ * S * S * D / 2 * 3.5 + 3 * 2 * S * H * (NQ + 2 * NKV) * D  # causal attn fwd+bwd (2.5x) + proj
    print(json.dumps({"kind": kind, "seq": S, "chunks": chunks if kind == "fpdt" else None,
                      "ms_fwd_bwd": round(dt * 1e3, 1), "TFLOPs": round(flops / dt / 1e12, 1),
                      "saved_for_backward_gib": round(held[0] / 2**30, 2),
                      "peak_extra_gib": round((torch.cuda.max_memory_allocated() - base) / 2**30, 2)}), flush=True)


def main():
    seqs = [int(s) for s in sys.argv[1].split(",")] if len(sys.argv) > 1 else [65536, 131072, 262144]
    chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    for S in seqs:
        for kind in ("plain", "fpdt"):
            try:
                run(kind, S, chunks)
            except torch.OutOfMemoryError as e:
                print(json.dumps({"kind": kind, "seq": S, "oom": str(e)[:120]}), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
