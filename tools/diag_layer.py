"""Per-op timing inside one Llama-3-8B decoder layer forward+backward (T=16384), events around each op."""
import torch
import torch.nn.functional as F
from hcache_deepspeed_amd.models import llama
from hcache_deepspeed_amd.ops.rope import rope_tables

cfg = llama.llama3_8b()
layer = llama.LlamaDecoderLayer(cfg).cuda().to(torch.bfloat16)
T, S = 16384, 4096
h = torch.randn(T, 4096, device="cuda", dtype=torch.bfloat16, requires_grad=True)
cos, sin = rope_tables(8192, 128, cfg.rope_theta, cfg.rope_scaling, device="cuda")
res = torch.randn_like(h)

def timed(name, fn, acc):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); out = fn(); e.record()
    acc.setdefault(name, []).append((s, e))
    return out

for it in range(8):
    acc = {}
    x, r = timed("norm1", lambda: layer.input_layernorm(h, res), acc)
    qkv = timed("qkv_gemm", lambda: layer.self_attn.qkv_proj(x), acc)
    from hcache_deepspeed_amd.ops.attention import qkv_attention
    o = timed("attn_fwd", lambda: qkv_attention(qkv.view(T, 48, 128), 32, 8, cos, sin, seq_len=S, causal=True), acc)
    a = timed("o_gemm", lambda: layer.self_attn.o_proj(o), acc)
    x2, r2 = timed("norm2", lambda: layer.post_attention_layernorm(a, r), acc)
    gu = timed("gate_up_gemm", lambda: layer.mlp.gate_up_proj(x2), acc)
    from hcache_deepspeed_amd.ops.activations import glu
    g = timed("glu", lambda: glu(gu, "silu"), acc)
    y = timed("down_gemm", lambda: layer.mlp.down_proj(g), acc)
    loss = (y.float().square().mean() + r2.float().square().mean())
    timed("backward", lambda: loss.backward(), acc)
    torch.cuda.synchronize()
    if it >= 5:
        print(" | ".join(f"{k} {sum(s.elapsed_time(e) for s, e in v):.2f}" for k, v in acc.items()), flush=True)
    layer.zero_grad(set_to_none=True)
    h.grad = None
