"""Kernel injection for ``init_inference``: swap HF building blocks for this framework's HIP kernels.

Reference parity: module_inject/replace_module.py (``replace_transformer_layer`` :183, ``generic_injection``
:88) with its per-architecture containers. The reference replaces whole layers with
``DeepSpeedTransformerInference``; here injection is done at the level of the blocks that have a HIP
kernel, which keeps every HF model's own cache / generate logic intact:

* ``*RMSNorm`` (Llama, Mistral, Mixtral, Qwen2, Gemma-style weight) -> :class:`FusedRMSNorm` (wave64 norm kernel)
* gated MLPs with ``gate_proj``/``up_proj``/``down_proj`` -> :class:`FusedGatedMLP` (one GEMM for gate|up +
  the gated-activation kernel)
* attention -> the ``hds_flash`` attention function (HIP FlashAttention for prefill, SDPA for the
  cached single-token decode whose causal alignment differs)
* optional weight-only INT8/INT4 quantization of every ``nn.Linear`` (:class:`QuantizedLinear`,
  reference inference/quantization).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import quantizer as Q
from ..ops.activations import glu
from ..ops.norm import rms_norm


class FusedRMSNorm(nn.Module):

    def __init__(self, weight, eps, offset=0.0, trainable=False):
        super().__init__()
        self.weight = nn.Parameter(weight.detach() + offset, requires_grad=trainable)
        self.eps = float(eps)

    def forward(self, x):
        shape = x.shape
        return rms_norm(x.reshape(-1, shape[-1]), self.weight, self.eps).view(shape)


class FusedGatedMLP(nn.Module):

    def __init__(self, gate, up, down, act="silu"):
        super().__init__()
        w = torch.cat([gate.weight.detach(), up.weight.detach()], 0)
        self.gate_up = nn.Linear(w.shape[1], w.shape[0], bias=False, device=w.device, dtype=w.dtype)
        self.gate_up.weight = nn.Parameter(w, requires_grad=False)
        self.down = down
        self.act = act

    def forward(self, x):
        shape = x.shape
        h = self.gate_up(x.reshape(-1, shape[-1]))
        return self.down(glu(h, self.act)).view(*shape[:-1], -1)


class QuantizedLinear(nn.Module):
    """Weight-only quantized linear: int8/int4 groups along the input dim (fused GEMV for decode, dequantize +
    GEMM for prefill)."""

    def __init__(self, linear, bits=8, group_size=128):
        super().__init__()
        w = linear.weight.detach()
        self.out_features, self.in_features = w.shape
        gs = group_size if self.in_features % group_size == 0 else self.in_features
        self.bits, self.group_size, self.dtype = bits, gs, w.dtype
        q, s, _ = Q.quantize(w.reshape(-1).contiguous(), gs, bits, True)
        self.register_buffer("qweight", q)
        self.register_buffer("scales", s)
        self.bias = linear.bias

    def forward(self, x):
        # decode (<= 8 rows): fused int8/int4 GEMV on the packed weight; prefill: dequantize + hipBLASLt
        return Q.int_linear(x, self.qweight, self.scales, self.out_features, self.in_features, self.group_size,
                            self.bits, self.bias)


def _act_name(mlp):
    fn = getattr(mlp, "act_fn", None)
    n = type(fn).__name__.lower() if fn is not None else "silu"
    if "silu" in n or "swish" in n:
        return "silu"
    if "gelu" in n:
        return "gelu_tanh" if "tanh" in n or "pytorch" in n else "gelu"
    if "relu" in n:
        return "relu"
    return None


def _hds_attention(module, query, key, value, attention_mask, scaling, dropout=0.0, **kwargs):
    """transformers AttentionInterface function: q [B,H,Sq,D], k/v [B,Hkv,Skv,D] -> ([B,Sq,H,D], None)."""
    from ..ops.attention import flash_attn
    B, H, Sq, D = query.shape
    Skv = key.shape[2]
    use_flash = (query.is_cuda and D == 128 and Sq == Skv and query.dtype == torch.bfloat16 and
                 (attention_mask is None or getattr(module, "is_causal", True)) and dropout == 0.0)
    if use_flash:
        o = flash_attn(query.transpose(1, 2), key.transpose(1, 2).contiguous(), value.transpose(1, 2).contiguous(),
                       causal=True, softmax_scale=scaling)
        return o, None
    rep = H // key.shape[1]
    k = key.repeat_interleave(rep, 1) if rep > 1 else key
    v = value.repeat_interleave(rep, 1) if rep > 1 else value
    mask = attention_mask[:, :, :, :Skv] if attention_mask is not None and attention_mask.dim() == 4 else None
    o = F.scaled_dot_product_attention(query, k, v, attn_mask=mask, is_causal=mask is None and Sq > 1 and Sq == Skv,
                                       scale=scaling)
    return o.transpose(1, 2).contiguous(), None


def register_attention():
    try:
        from transformers import AttentionInterface
        AttentionInterface.register("hds_fused_attn", _hds_attention)
        return True
    except Exception:  # noqa: BLE001
        return False


def inject(model, quant=None, trainable=False, fuse_mlp=True):
    """In-place kernel injection; returns the number of replaced blocks. This framework's own modules are
    already fused and are left alone. ``trainable``/``fuse_mlp=False`` keep parameter names and grads (used
    by the hybrid engine before ZeRO partitions the model)."""
    n = 0
    for parent in list(model.modules()):
        for cname, child in list(parent.named_children()):
            cls = type(child).__name__
            if type(child).__module__.startswith("hcache_deepspeed_amd"):
                continue
            if cls.endswith("RMSNorm") and hasattr(child, "weight"):
                eps = getattr(child, "variance_epsilon", getattr(child, "eps", 1e-6))
                offset = 1.0 if "Gemma" in cls else 0.0
                setattr(parent, cname, FusedRMSNorm(child.weight, eps, offset, trainable))
                n += 1
            elif fuse_mlp and all(hasattr(child, a) for a in ("gate_proj", "up_proj", "down_proj")) and \
                    getattr(child.gate_proj, "bias", None) is None and _act_name(child) is not None:
                setattr(parent, cname, FusedGatedMLP(child.gate_proj, child.up_proj, child.down_proj, _act_name(child)))
                n += 1
    cfg = getattr(model, "config", None)
    if cfg is not None and hasattr(cfg, "_attn_implementation") and register_attention():
        try:
            cfg._attn_implementation = "hds_fused_attn"
            for sub in model.modules():
                sc = getattr(sub, "config", None)
                if sc is not None and hasattr(sc, "_attn_implementation"):
                    sc._attn_implementation = "hds_fused_attn"
            n += 1
        except Exception:  # noqa: BLE001
            pass
    if quant is not None and quant.enabled:
        for parent in list(model.modules()):
            for cname, child in list(parent.named_children()):
                if isinstance(child, nn.Linear) and child.weight.is_cuda and "lm_head" not in cname:
                    setattr(parent, cname, QuantizedLinear(child, quant.bits, quant.group_size))
                    n += 1
    return n
