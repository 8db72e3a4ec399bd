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
* ``nn.LayerNorm`` (GPT-2, GPT-J, GPT-Neo, GPT-NeoX, OPT, BLOOM, BERT) -> :class:`FusedLayerNorm`
* non-gated MLPs: the up-projection + activation pair (GPT-2/GPT-Neo ``c_fc``+``act``, GPT-J ``fc_in``+``act``,
  GPT-NeoX ``dense_h_to_4h``+``act``, BLOOM ``dense_h_to_4h``+``gelu_impl``, OPT ``fc1``+``activation_fn``,
  BERT ``intermediate.dense``+``intermediate_act_fn``) -> :class:`LinearBiasAct` (bias-free GEMM + one fused
  bias+activation kernel); the activation attribute becomes identity so each model keeps its own forward
  (dropout, residual handling, caches). This covers the reference's per-architecture containers
  (module_inject/containers/{gpt2,gptj,gptneo,gptneox,opt,bloom,bert}.py) without a policy per model.
* optional weight-only INT8/INT4 quantization of every ``nn.Linear`` (:class:`QuantizedLinear`,
  reference inference/quantization).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import quantizer as Q
from ..ops.activations import bias_act, glu
from ..ops.norm import layer_norm, rms_norm


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


class FusedLayerNorm(nn.Module):

    def __init__(self, ln, trainable=False):
        super().__init__()
        self.weight = nn.Parameter(ln.weight.detach().clone(), requires_grad=trainable)
        self.bias = nn.Parameter(ln.bias.detach().clone(), requires_grad=trainable) if ln.bias is not None else None
        self.eps = float(ln.eps)

    def forward(self, x):
        shape = x.shape
        return layer_norm(x.reshape(-1, shape[-1]), self.weight, self.bias, self.eps).view(shape)


class LinearBiasAct(nn.Module):
    """act(x @ W^T + b) as one hipBLASLt GEMM plus the fused bias+activation kernel. ``conv1d`` accepts the
    GPT-2 ``Conv1D`` layout (weight [in, out])."""

    def __init__(self, linear, act, conv1d=False):
        super().__init__()
        w = linear.weight.detach()
        w = w.t().contiguous() if conv1d else w
        self.weight = nn.Parameter(w, requires_grad=False)
        b = linear.bias
        self.bias = nn.Parameter(b.detach(), requires_grad=False) if b is not None else None
        self.act = act

    def forward(self, x):
        from ..ops.gemv import linear  # decode steps (<= 8 tokens) on the HIP GEMV
        return bias_act(linear(x, self.weight), self.bias, self.act)


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


# HF activation class -> fused kernel activation (transformers/activations.py names)
_ACT_CLASSES = {
    "silu": "silu", "siluactivation": "silu", "swish": "silu",
    "newgeluactivation": "gelu_tanh", "fastgeluactivation": "gelu_tanh", "pytorchgelutanh": "gelu_tanh",
    "gelutanh": "gelu_tanh", "bloomgelu": "gelu_tanh", "gelupytorchtanh": "gelu_tanh",
    "geluactivation": "gelu", "gelu": "gelu", "relu": "relu",
}


def _act_of(fn):
    if fn is None:
        return None
    name = type(fn).__name__.lower()
    if name == "gelu" and getattr(fn, "approximate", "none") == "tanh":
        return "gelu_tanh"
    if name == "geluactivation" and getattr(fn, "act", F.gelu) is not F.gelu:
        return None  # python-erf variant: same math, keep HF's module
    if name in ("function", "builtin_function_or_method"):
        return {F.silu: "silu", F.relu: "relu", F.gelu: "gelu"}.get(fn)
    return _ACT_CLASSES.get(name)


def _act_name(mlp):
    fn = getattr(mlp, "act_fn", None)
    return "silu" if fn is None else _act_of(fn)


# (up-projection attribute, activation attribute) pairs of non-gated MLP owners
_UP_ACT = (("c_fc", "act"), ("fc_in", "act"), ("dense_h_to_4h", "act"), ("dense_h_to_4h", "gelu_impl"),
           ("fc1", "activation_fn"), ("dense", "intermediate_act_fn"))


class _Identity(nn.Module):

    def forward(self, x, *args, **kwargs):
        return x


def _inject_up_act(module):
    for up_name, act_name in _UP_ACT:
        up = getattr(module, up_name, None)
        if up is None or isinstance(up, LinearBiasAct) or not hasattr(module, act_name):
            continue
        act = _act_of(getattr(module, act_name))
        conv1d = type(up).__name__ == "Conv1D"
        if act is None or not (isinstance(up, nn.Linear) or conv1d):
            continue
        n_out = up.weight.shape[1] if conv1d else up.weight.shape[0]
        if n_out % 8:
            continue
        setattr(module, up_name, LinearBiasAct(up, act, conv1d))
        setattr(module, act_name, _Identity())
        return True
    return False


def _hds_attention(module, query, key, value, attention_mask, scaling, dropout=0.0, **kwargs):
    """transformers AttentionInterface function: q [B,H,Sq,D], k/v [B,Hkv,Skv,D] -> ([B,Sq,H,D], None)."""
    from ..ops.attention import flash_attn, head_dim_supported
    B, H, Sq, D = query.shape
    Skv = key.shape[2]
    causal = bool(getattr(module, "is_causal", True))
    use_flash = (query.is_cuda and head_dim_supported(D) and Sq == Skv and query.dtype == torch.bfloat16 and causal
                 and dropout == 0.0)
    if use_flash:
        o = flash_attn(query.transpose(1, 2), key.transpose(1, 2).contiguous(), value.transpose(1, 2).contiguous(),
                       causal=True, softmax_scale=scaling)
        return o, None
    from ..ops.decode_attention import decode_attention, decode_supported, sdpa_gqa
    mask = attention_mask[:, :, :, :Skv] if attention_mask is not None and attention_mask.dim() == 4 else None
    if Sq == 1 and dropout == 0.0 and decode_supported(query[:, :, 0], key):
        # generation step: one query row against the cache, GQA served from the kv heads directly
        bias = None
        if mask is not None:
            m = mask[:, 0, -1, :]
            bias = m if m.is_floating_point() else torch.zeros(m.shape, device=m.device).masked_fill(~m, float("-inf"))
        o = decode_attention(query[:, :, 0], key, value, scaling, bias=bias)
        return o[:, None], None
    o = sdpa_gqa(query, key, value, mask=mask, is_causal=causal and mask is None and Sq > 1 and Sq == Skv,
                 scale=scaling)
    return o.transpose(1, 2).contiguous(), None


def _uses_attention_interface(model):
    """Only families whose attention dispatches through transformers' AttentionInterface get the fused
    function; the others (GPT-J, GPT-Neo, BLOOM's ALiBi path) build their masks for their own attention."""
    import sys
    mod = sys.modules.get(type(model).__module__)
    return mod is not None and hasattr(mod, "ALL_ATTENTION_FUNCTIONS")


def register_attention():
    try:
        from transformers import AttentionInterface
        AttentionInterface.register("hds_fused_attn", _hds_attention)
        try:  # masks for our implementation: the SDPA form (None when plain causal -> the flash path)
            from transformers.masking_utils import AttentionMaskInterface, sdpa_mask
            AttentionMaskInterface.register("hds_fused_attn", sdpa_mask)
        except ImportError:
            pass
        return True
    except Exception:  # noqa: BLE001
        return False


def inject(model, quant=None, trainable=False, fuse_mlp=True):
    """In-place kernel injection; returns the number of replaced blocks. This framework's own modules are
    already fused and are left alone. ``trainable``/``fuse_mlp=False`` keep parameter names and grads (used
    by the hybrid engine before ZeRO partitions the model)."""
    n = 0
    if not trainable:
        # family containers that replace whole blocks come first (they read the original LayerNorm weights)
        from .megatron import inject_internlm, inject_megatron_layers
        n += inject_megatron_layers(model) + inject_internlm(model)
        from .diffusers import inject_attention_processors
        n += inject_attention_processors(model)  # diffusers-style Attention modules (UNet / VAE blocks)
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
            elif isinstance(child, nn.LayerNorm) and child.elementwise_affine and \
                    len(child.normalized_shape) == 1 and child.normalized_shape[0] % 8 == 0:
                setattr(parent, cname, FusedLayerNorm(child, trainable))
                n += 1
            elif fuse_mlp and all(hasattr(child, a) for a in ("gate_proj", "up_proj", "down_proj")) and \
                    getattr(child.gate_proj, "bias", None) is None and _act_name(child) is not None:
                setattr(parent, cname, FusedGatedMLP(child.gate_proj, child.up_proj, child.down_proj, _act_name(child)))
                n += 1
            elif fuse_mlp and not trainable and _inject_up_act(child):
                n += 1
    cfg = getattr(model, "config", None)
    if cfg is not None and hasattr(cfg, "_attn_implementation") and _uses_attention_interface(model) and \
            register_attention():
        try:
            cfg._attn_implementation = "hds_fused_attn"
            for sub in model.modules():
                sc = getattr(sub, "config", None)
                if sc is not None and hasattr(sc, "_attn_implementation"):
                    sc._attn_implementation = "hds_fused_attn"
            n += 1
        except Exception:  # noqa: BLE001
            pass
    elif not trainable:
        from .containers import inject_attention_containers
        n += inject_attention_containers(model)  # GPT-J / GPT-Neo / BLOOM: family attention containers
    if quant is not None and quant.enabled:
        for parent in list(model.modules()):
            for cname, child in list(parent.named_children()):
                if isinstance(child, nn.Linear) and child.weight.is_cuda and "lm_head" not in cname:
                    setattr(parent, cname, QuantizedLinear(child, quant.bits, quant.group_size))
                    n += 1
    return n
