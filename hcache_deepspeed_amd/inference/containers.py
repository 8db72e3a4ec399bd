"""Per-family attention containers for HF models whose attention does not dispatch through transformers'
AttentionInterface (GPT-J, GPT-Neo, BLOOM): their attention core is swapped, in place and weight-preserving, for
this framework's kernels.

Reference parity: deepspeed/module_inject/containers/{gptj,gptneo,bloom}.py (policy classes mapping each family's
attention onto the fused inference kernels: rotary / local-window / ALiBi variants) and the KV-cache
``softmax_context`` path (csrc/transformer/inference/csrc/pt_binding.cpp:1969-2036).

What runs:
  * a generation step (one query row) -> csrc/kernels/decode_attn.hip over the HF cache tensors, with the padding
    mask row, GPT-Neo's local window and BLOOM's ALiBi slopes applied in-kernel;
  * a prefill whose mask is plain causal (no padding) -> the HIP FlashAttention kernel (sliding window for
    GPT-Neo local layers);
  * anything else (padded prefill, ALiBi prefill) -> fused SDPA with one combined additive mask.
The projections, rotary embedding, cache update and output projection stay the model's own code.
"""
import math
import types

import torch
import torch.nn.functional as F


def _window_bias(Sq, Skv, window, device):
    """Additive [Sq, Skv] bias keeping keys j with q - window < j <= q (q = Skv - Sq + row)."""
    qpos = torch.arange(Skv - Sq, Skv, device=device)[:, None]
    kpos = torch.arange(Skv, device=device)[None, :]
    keep = (kpos <= qpos) & (kpos > qpos - window)
    return torch.zeros(Sq, Skv, device=device).masked_fill(~keep, float("-inf"))


def _is_plain_causal(mask, Sq, Skv):
    """True when an additive / boolean 4-D mask hides no key beyond causality (no padding anywhere)."""
    if mask is None:
        return True
    if Sq != Skv or mask.dim() != 4:
        return False
    first_col = mask[..., :, 0]
    last_row = mask[..., -1, :]
    if mask.dtype == torch.bool:
        return bool(first_col.all()) and bool(last_row.all())
    return bool((first_col == 0).all()) and bool((last_row == 0).all())


def alibi_slopes(num_heads, device="cpu"):
    """The ALiBi head slopes of Press et al. (BLOOM's build_alibi_tensor), as a float32 [H] tensor."""
    closest = 2**math.floor(math.log2(num_heads))
    base = 2**(-(2**-(math.log2(closest) - 3)))
    slopes = [base**(i + 1) for i in range(closest)]
    if closest != num_heads:
        extra = 2**(-(2**-(math.log2(2 * closest) - 3)))
        slopes += [extra**(i + 1) for i in range(0, 2 * (num_heads - closest), 2)]
    return torch.tensor(slopes, dtype=torch.float32, device=device)


def fused_core_attention(q, k, v, mask=None, scale=1.0, window=0, slopes=None):
    """q [B, H, Sq, D], k/v [B, Hkv, Skv, D], mask additive/bool [B, 1|H, Sq, Skv] or None -> [B, H, Sq, D]."""
    from ..ops.attention import flash_attn, head_dim_supported
    from ..ops.decode_attention import decode_attention, decode_supported
    B, H, Sq, D = q.shape
    Skv = k.shape[2]
    dt = q.dtype
    if mask is not None and mask.dtype == torch.bool:
        mask = torch.zeros(mask.shape, device=q.device, dtype=torch.float32).masked_fill(~mask, float("-inf"))
    if Sq == 1 and decode_supported(q[:, :, 0], k):
        bias = None
        if mask is not None:
            bias = mask[:, 0, -1, :].float()
        if window and Skv > window:
            wb = torch.zeros(Skv, device=q.device).masked_fill(torch.arange(Skv, device=q.device) <= Skv - 1 - window,
                                                               float("-inf"))
            bias = wb[None].expand(B, Skv) if bias is None else bias + wb[None]
        o = decode_attention(q[:, :, 0], k.to(dt), v.to(dt), scale, bias=bias, alibi=slopes)
        return o[:, :, None]
    if (slopes is None and q.is_cuda and dt == torch.bfloat16 and head_dim_supported(D) and
            _is_plain_causal(mask, Sq, Skv)):
        o = flash_attn(q.transpose(1, 2), k.transpose(1, 2).contiguous(), v.transpose(1, 2).contiguous(), causal=True,
                       softmax_scale=scale, window=window)
        return o.transpose(1, 2)
    bias = torch.zeros(Sq, Skv, device=q.device, dtype=torch.float32)
    if window:
        bias = _window_bias(Sq, Skv, window, q.device)
    elif mask is None:
        bias = _window_bias(Sq, Skv, Skv + 1, q.device)  # plain causal
    bias = bias[None, None]
    if mask is not None:
        bias = bias + mask[..., :Skv].float()
    if slopes is not None:
        rel = (torch.arange(Skv, device=q.device) - (Skv - 1)).float()
        bias = bias + slopes.to(q.device)[None, :, None, None] * rel[None, None, None, :]
    o = F.scaled_dot_product_attention(q.float(), k.float(), v.float(), attn_mask=bias, scale=scale,
                                       enable_gqa=k.shape[1] != H)
    return o.to(dt)


# ---- GPT-J ---------------------------------------------------------------------------------------------
def _gptj_attn(self, query, key, value, attention_mask=None):
    scale = 1.0 / float(self.scale_attn)
    return fused_core_attention(query, key, value, attention_mask, scale=scale), None


# ---- GPT-Neo (no 1/sqrt(d) scaling; local layers: sliding window) --------------------------------------
def _gptneo_attn(self, query, key, value, attention_mask=None):
    window = self.config.window_size if getattr(self, "attention_type", "global") == "local" else 0
    return fused_core_attention(query, key, value, attention_mask, scale=1.0, window=window), None


# ---- BLOOM (fused QKV, ALiBi) --------------------------------------------------------------------------
def _bloom_forward(self, hidden_states, residual, alibi, attention_mask, layer_past=None, use_cache=False,
                   output_attentions=False, **kwargs):
    fused_qkv = self.query_key_value(hidden_states)
    q, k, v = self._reshape(fused_qkv)
    if layer_past is not None:
        k, v = layer_past.update(k, v, self.layer_idx)
    if getattr(self, "_hds_slopes", None) is None or self._hds_slopes.device != q.device:
        self._hds_slopes = alibi_slopes(self.num_heads, q.device)
    ctx = fused_core_attention(q, k, v, attention_mask, scale=float(self.inv_norm_factor), slopes=self._hds_slopes)
    B, H, Sq, D = ctx.shape
    ctx = ctx.transpose(1, 2).reshape(B, Sq, H * D)
    out = self.dense(ctx)
    out = F.dropout(out, p=self.hidden_dropout, training=self.training) + residual
    return out, None


_CONTAINERS = {
    "GPTJAttention": ("_attn", _gptj_attn),
    "GPTNeoSelfAttention": ("_attn", _gptneo_attn),
    "BloomAttention": ("forward", _bloom_forward),
}


def inject_attention_containers(model):
    """Swap the attention core of every supported family module in ``model``; returns how many were replaced."""
    n = 0
    for m in model.modules():
        spec = _CONTAINERS.get(type(m).__name__)
        if spec is None or getattr(m, "_hds_container", False):
            continue
        name, fn = spec
        setattr(m, name, types.MethodType(fn, m))
        m._hds_container = True
        n += 1
    return n
