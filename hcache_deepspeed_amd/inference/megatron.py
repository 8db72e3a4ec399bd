"""Megatron-GPT, Megatron-GPT-MoE and InternLM injection containers.

Reference parity: deepspeed/module_inject/containers/megatron_gpt.py (``MegatronLayerPolicy``: the
``ParallelTransformerLayer`` of Megatron-LM, version 0 ``attention.*`` / version 1 ``self_attention.*``, weights
``query_key_value`` / ``dense`` / ``mlp.dense_h_to_4h`` / ``mlp.dense_4h_to_h`` / the two LayerNorms, converted
into the fused ``DeepSpeedGPTInference`` block), megatron_gpt_moe.py (same block with the Megatron-DeepSpeed MoE
MLP -- ``mlp.deepspeed_moe.experts`` -- kept as the expert path) and internlm.py (``InternLMLayerPolicy``: a
LLaMA-style block with biased q/k/v/o projections; InternLM2's fused ``wqkv`` / ``wo`` layout with GQA).

MI355X design: the converted block runs this framework's HIP kernels end to end -- fused LayerNorm (with the
residual add folded into the second norm), one qkv GEMM whose output is split with Megatron's per-head
[heads, 3, head_dim] interleave, causal FlashAttention (prefill) or split-K decode attention over the block's own
KV cache (incremental decoding), the o projection, bias+GeLU fused into one kernel after the h->4h GEMM, and the
4h->h GEMM. Megatron's layers are sequence-first ([s, b, h]); the block keeps that layout at its boundary.
The InternLM container swaps the attention module's forward for one on the same kernels (biased projections,
rotary from the module's own ``rotary_emb``, KV cache as a (k, v) tuple like the remote code expects).
Megatron-LM and the InternLM remote code are not dependencies: layers are recognised by their attribute layout.
"""
import math
import types

import torch
import torch.nn as nn
import torch.nn.functional as F


def _megatron_attn(layer):
    """(attention module, version) of a Megatron ParallelTransformerLayer-shaped module, or (None, None)."""
    for name, ver in (("self_attention", 1), ("attention", 0)):
        a = getattr(layer, name, None)
        if a is not None and hasattr(a, "query_key_value") and hasattr(a, "dense"):
            return a, ver
    return None, None


def is_megatron_layer(m):
    # HF GPT-NeoX / BLOOM blocks share the attribute names; they have their own containers (inference/containers.py)
    if type(m).__module__.startswith("transformers."):
        return False
    a, _ = _megatron_attn(m)
    return (a is not None and hasattr(m, "input_layernorm") and hasattr(m, "post_attention_layernorm")
            and hasattr(m, "mlp"))


def _moe_experts(mlp):
    moe = getattr(mlp, "deepspeed_moe", None)
    return moe is not None and hasattr(moe, "experts")


class DSMegatronGPTBlock(nn.Module):
    """Fused inference block converted from a Megatron GPT layer (see module docstring)."""

    def __init__(self, layer):
        super().__init__()
        attn, self.version = _megatron_attn(layer)
        self.heads = int(getattr(attn, "num_attention_heads_per_partition", None)
                         or getattr(attn, "num_attention_heads", None) or getattr(layer, "num_attention_heads"))
        ln1, ln2 = layer.input_layernorm, layer.post_attention_layernorm
        self.eps = float(getattr(ln1, "eps", 1e-5))
        wd = lambda t: None if t is None else t.detach()  # noqa: E731
        self.ln1_w, self.ln1_b = wd(ln1.weight), wd(getattr(ln1, "bias", None))
        self.ln2_w, self.ln2_b = wd(ln2.weight), wd(getattr(ln2, "bias", None))
        self.qkv_w, self.qkv_b = wd(attn.query_key_value.weight), wd(getattr(attn.query_key_value, "bias", None))
        self.o_w, self.o_b = wd(attn.dense.weight), wd(getattr(attn.dense, "bias", None))
        self.moe = layer.mlp if _moe_experts(layer.mlp) else None
        if self.moe is None:
            self.h4_w, self.h4_b = wd(layer.mlp.dense_h_to_4h.weight), wd(getattr(layer.mlp.dense_h_to_4h, "bias", None))
            self.o4_w, self.o4_b = wd(layer.mlp.dense_4h_to_h.weight), wd(getattr(layer.mlp.dense_4h_to_h, "bias", None))
        self.apply_residual_post_ln = bool(getattr(layer, "apply_residual_connection_post_layernorm", False))
        # incremental-decoding KV cache: preallocated [b, heads, capacity, d] buffers, grown by doubling; a decode
        # token is written in place by the HIP kv_append kernel (one launch for k and v), not by concatenation
        self.kc = self.vc = None
        self.kv_len = 0

    def reset_cache(self):
        self.kc = self.vc = None
        self.kv_len = 0

    @property
    def kv(self):
        """(k, v) views [b, heads, t, d] of the cached tokens, or None."""
        if self.kc is None:
            return None
        return self.kc[:, :, :self.kv_len], self.vc[:, :, :self.kv_len]

    def _cache_append(self, k, v):
        b, nh, s, d = k.shape
        t0, need = self.kv_len, self.kv_len + s
        if self.kc is None or need > self.kc.shape[2] or self.kc.shape[0] != b:
            cap = max(need, 2 * (self.kc.shape[2] if self.kc is not None else 0), 256)
            kc, vc = k.new_empty(b, nh, cap, d), v.new_empty(b, nh, cap, d)
            if t0:
                kc[:, :, :t0].copy_(self.kc[:, :, :t0])
                vc[:, :, :t0].copy_(self.vc[:, :, :t0])
            self.kc, self.vc = kc, vc
        if s == 1 and k.is_cuda:
            from ..ops.decode_attention import kv_append
            kv_append(k[:, :, 0], v[:, :, 0], self.kc, self.vc, torch.tensor([t0], device=k.device, dtype=torch.int64))
        else:
            self.kc[:, :, t0:need].copy_(k)
            self.vc[:, :, t0:need].copy_(v)
        self.kv_len = need
        return self.kc[:, :, :need], self.vc[:, :, :need]

    def _ln(self, x, w, b, residual=None):
        from ..ops.norm import layer_norm
        return layer_norm(x, w, b, self.eps, residual=residual)

    def _attention(self, x, s, b, use_cache):
        from .containers import fused_core_attention
        nh = self.heads
        qkv = F.linear(x, self.qkv_w, self.qkv_b)  # [s*b, 3h], Megatron layout [heads, 3, d] per token
        d = qkv.shape[-1] // (3 * nh)
        qkv = qkv.view(s, b, nh, 3, d)
        q, k, v = (qkv[:, :, :, i].permute(1, 2, 0, 3) for i in range(3))  # [b, nh, s, d]
        if use_cache:
            k, v = self._cache_append(k, v)
        else:
            k, v = k.contiguous(), v.contiguous()
        o = fused_core_attention(q.contiguous(), k, v, None, scale=1.0 / math.sqrt(d))
        return o.permute(2, 0, 1, 3).reshape(s * b, nh * d)  # [s*b, h]

    @torch.no_grad()
    def forward(self, hidden_states, attention_mask=None, *args, use_cache=False, **kwargs):
        from ..ops.activations import bias_act
        s, b, H = hidden_states.shape
        x = hidden_states.reshape(s * b, H)
        h = self._ln(x, self.ln1_w, self.ln1_b)
        a = F.linear(self._attention(h, s, b, use_cache), self.o_w, self.o_b)
        # Megatron: the residual around attention is the layer input, or the first norm's output with
        # apply_residual_connection_post_layernorm; around the MLP it is the norm input / output likewise
        res = h if self.apply_residual_post_ln else x
        h2, x1 = self._ln(a, self.ln2_w, self.ln2_b, residual=res)  # x1 = residual + attention, h2 = LN(x1)
        mlp_res = h2 if self.apply_residual_post_ln else x1
        if self.moe is not None:
            mo = self.moe(h2.view(s, b, H))
            mo = mo[0] if isinstance(mo, tuple) else mo
            out = mlp_res + mo.reshape(s * b, H)
        else:
            f = bias_act(F.linear(h2, self.h4_w), self.h4_b, "gelu")
            out = mlp_res + F.linear(f, self.o4_w, self.o4_b)
        return out.view(s, b, H)


def inject_megatron_layers(model):
    """Replace every Megatron GPT (or GPT-MoE) layer under ``model`` by ``DSMegatronGPTBlock``; returns the count."""
    n = 0
    for parent in list(model.modules()):
        for cname, child in list(parent.named_children()):
            if not isinstance(child, DSMegatronGPTBlock) and is_megatron_layer(child):
                setattr(parent, cname, DSMegatronGPTBlock(child))
                n += 1
    return n


# ---- InternLM -------------------------------------------------------------------------------------------------
def _rotate_half(x):
    a, b = x.chunk(2, dim=-1)
    return torch.cat((-b, a), dim=-1)


def _internlm_attn_forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_value=None,
                           output_attentions=False, use_cache=False, **kwargs):
    from .containers import fused_core_attention
    B, S, _ = hidden_states.shape
    nh, d = self.num_heads, self.head_dim
    q = self.q_proj(hidden_states).view(B, S, nh, d).transpose(1, 2)
    k = self.k_proj(hidden_states).view(B, S, nh, d).transpose(1, 2)
    v = self.v_proj(hidden_states).view(B, S, nh, d).transpose(1, 2)
    kv_len = S + (past_key_value[0].shape[-2] if past_key_value is not None else 0)
    cos, sin = self.rotary_emb(v, seq_len=kv_len)
    if position_ids is None:
        position_ids = torch.arange(kv_len - S, kv_len, device=q.device)[None].expand(B, S)
    cos = cos.squeeze(1).squeeze(0)[position_ids].unsqueeze(1).to(q.dtype)  # [B, 1, S, d]
    sin = sin.squeeze(1).squeeze(0)[position_ids].unsqueeze(1).to(q.dtype)
    q = q * cos + _rotate_half(q) * sin
    k = k * cos + _rotate_half(k) * sin
    if past_key_value is not None:
        k = torch.cat([past_key_value[0], k], 2)
        v = torch.cat([past_key_value[1], v], 2)
    past = (k, v) if use_cache else None
    o = fused_core_attention(q, k, v, attention_mask, scale=1.0 / math.sqrt(d))
    o = self.o_proj(o.transpose(1, 2).reshape(B, S, nh * d))
    return o, None, past


def _internlm2_attn_forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_value=None,
                            output_attentions=False, use_cache=False, **kwargs):
    """InternLM2 attention: ONE fused ``wqkv`` projection laid out per kv head as [q_per_kv query heads, k, v]
    (x head_dim), GQA, ``wo`` output; same kernels as InternLM (reference containers/internlm.py)."""
    from .containers import fused_core_attention
    B, S, _ = hidden_states.shape
    nh, d = self.num_heads, self.head_dim
    nkv = int(getattr(self, "num_key_value_heads", nh))
    g = nh // nkv
    qkv = self.wqkv(hidden_states).view(B, S, nkv, g + 2, d)
    q = qkv[:, :, :, :g].reshape(B, S, nh, d).transpose(1, 2)
    k = qkv[:, :, :, g].transpose(1, 2)
    v = qkv[:, :, :, g + 1].transpose(1, 2)
    kv_len = S + (past_key_value[0].shape[-2] if past_key_value is not None else 0)
    cos, sin = self.rotary_emb(v, seq_len=kv_len)
    if position_ids is None:
        position_ids = torch.arange(kv_len - S, kv_len, device=q.device)[None].expand(B, S)
    cos = cos.squeeze(1).squeeze(0)[position_ids].unsqueeze(1).to(q.dtype)
    sin = sin.squeeze(1).squeeze(0)[position_ids].unsqueeze(1).to(q.dtype)
    q = q * cos + _rotate_half(q) * sin
    k = k * cos + _rotate_half(k) * sin
    if past_key_value is not None:
        k = torch.cat([past_key_value[0], k], 2)  # the remote code's cache contract: a (k, v) tuple returned
        v = torch.cat([past_key_value[1], v], 2)
    past = (k, v) if use_cache else None
    o = fused_core_attention(q, k.contiguous(), v.contiguous(), attention_mask, scale=1.0 / math.sqrt(d))
    o = self.wo(o.transpose(1, 2).reshape(B, S, nh * d))
    return o, None, past


def _is_internlm_attention(m):
    return type(m).__name__ in ("InternLMAttention", "InternLM2Attention") and \
        all(hasattr(m, a) for a in ("q_proj", "k_proj", "v_proj", "o_proj", "rotary_emb", "num_heads", "head_dim"))


def _is_internlm2_attention(m):
    return type(m).__name__ == "InternLM2Attention" and \
        all(hasattr(m, a) for a in ("wqkv", "wo", "rotary_emb", "num_heads", "head_dim"))


def inject_internlm(model):
    n = 0
    for m in model.modules():
        if getattr(m, "_hds_container", False):
            continue
        if _is_internlm2_attention(m):
            m.forward = types.MethodType(_internlm2_attn_forward, m)
        elif _is_internlm_attention(m):
            m.forward = types.MethodType(_internlm_attn_forward, m)
        else:
            continue
        m._hds_container = True
        n += 1
    return n
