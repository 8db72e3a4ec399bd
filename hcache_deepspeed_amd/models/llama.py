"""Llama-family causal LM (Llama-2/3, Mistral-style sliding window) built on the HIP op layer.

Training-side layout choices (MI355X-first):
* one fused QKV projection (``qkv_proj.weight`` = [(Hq + 2*Hkv) * D, H]) whose output is consumed
  in place by RoPE + FlashAttention (ops/attention.qkv_attention) -- no split/transpose copies;
* one fused gate|up projection ([2*I, H]) + the HIP SwiGLU kernel;
* pre-norm residual stream with the residual add fused into the next RMSNorm kernel;
* LM head + cross-entropy fused and chunked (never materialises [T, 128256] logits);
* ``model.layers`` is an ``nn.ModuleList`` -> each decoder block is one ZeRO-3 fetch unit.

HF checkpoint names (q_proj/k_proj/v_proj, gate_proj/up_proj) are converted by
:func:`convert_hf_state_dict`. Reference parity: the HF Llama model the reference trains through
``deepspeed.initialize`` and inference/v2/model_implementations/llama_v2 (serving).
"""
import math
import os
from dataclasses import asdict, dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activations import glu
from ..ops.attention import qkv_attention
from ..ops.cross_entropy import fused_linear_cross_entropy
from ..ops.norm import RMSNorm
from ..ops.rope import rope_tables
from ..runtime.activation_checkpointing.checkpointing import checkpoint as _ckpt


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: Optional[int] = None
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    sliding_window: int = 0
    hidden_act: str = "silu"
    initializer_range: float = 0.02
    model_type: str = "llama"

    def __post_init__(self):
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads

    def to_dict(self):
        return asdict(self)

    @staticmethod
    def from_dict(d):
        keys = LlamaConfig.__dataclass_fields__.keys()
        return LlamaConfig(**{k: v for k, v in d.items() if k in keys})

    def num_params(self, include_embedding=True):
        H, I, L, V = self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size
        D, Hq, Hkv = self.head_dim, self.num_attention_heads, self.num_key_value_heads
        per_layer = H * (Hq + 2 * Hkv) * D + Hq * D * H + 3 * H * I + 2 * H
        n = L * per_layer + H
        if include_embedding:
            n += V * H * (1 if self.tie_word_embeddings else 2)
        return n

    def flops_per_token(self, seq_len):
        """Training FLOPs/token (fwd+bwd, no recompute): 6N + 12*L*H*S (PaLM convention, matmul weights only)."""
        return 6 * self.num_params(include_embedding=False) + 6 * self.vocab_size * self.hidden_size + \
            12 * self.num_hidden_layers * self.hidden_size * seq_len

    def flops_per_token_causal(self, seq_len):
        """The same with the attention FLOPs a causal kernel actually performs: each query attends to ~half the keys
        ((S + 1) / 2 on average), so the score and P.V terms are 6*L*H*(S+1) instead of 12*L*H*S."""
        return 6 * self.num_params(include_embedding=False) + 6 * self.vocab_size * self.hidden_size + \
            6 * self.num_hidden_layers * self.hidden_size * (seq_len + 1)


def llama3_8b(**kw):
    return LlamaConfig(**kw)


def llama3_70b(**kw):
    d = dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
             num_key_value_heads=8)
    d.update(kw)
    return LlamaConfig(**d)


def llama2_7b(**kw):
    d = dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32, num_attention_heads=32,
             num_key_value_heads=32, rope_theta=10000.0, rms_norm_eps=1e-6, max_position_embeddings=4096)
    d.update(kw)
    return LlamaConfig(**d)


def mistral_7b(**kw):
    d = dict(vocab_size=32000, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
             num_key_value_heads=8, rope_theta=10000.0, sliding_window=4096, max_position_embeddings=32768,
             model_type="mistral")
    d.update(kw)
    return LlamaConfig(**d)


def tiny(**kw):
    d = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=2,
             num_key_value_heads=1, head_dim=128, max_position_embeddings=1024)
    d.update(kw)
    return LlamaConfig(**d)


def tiny_sp(**kw):
    """Tiny model whose 16 q / 8 kv heads split evenly over up to 8 Ulysses ranks (CPU dry runs of the
    sequence-parallel bench)."""
    d = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=16,
             num_key_value_heads=8, head_dim=16, max_position_embeddings=4096)
    d.update(kw)
    return LlamaConfig(**d)


PRESETS = {"llama3-8b": llama3_8b, "llama3-70b": llama3_70b, "llama2-7b": llama2_7b, "mistral-7b": mistral_7b,
           "tiny": tiny, "tiny-sp": tiny_sp}


class _Linear(nn.Linear):
    """nn.Linear with the model's init (normal(0, std)), bias-free by default."""

    def __init__(self, in_f, out_f, bias=False, std=0.02, **kw):
        self._std = std
        super().__init__(in_f, out_f, bias=bias, **kw)

    def reset_parameters(self):
        nn.init.normal_(self.weight, std=self._std)
        if self.bias is not None:
            nn.init.zeros_(self.bias)


class _Embedding(nn.Embedding):

    def __init__(self, n, d, std=0.02, **kw):
        self._std = std
        super().__init__(n, d, **kw)

    def reset_parameters(self):
        nn.init.normal_(self.weight, std=self._std)


def _fuse_hf_keys(parts, fused):
    """load_state_dict pre-hook: accept HF / reference parameter names (separate q/k/v and gate/up projections)
    for this model's fused GEMM weights, so HF and DeepSpeed state dicts load directly."""

    def hook(state_dict, prefix, *args):
        for kind in ("weight", "bias"):
            keys = [f"{prefix}{p}.{kind}" for p in parts]
            if all(k in state_dict for k in keys):
                state_dict[f"{prefix}{fused}.{kind}"] = torch.cat([state_dict.pop(k) for k in keys], 0)

    return hook


class LlamaAttention(nn.Module):

    def __init__(self, cfg: LlamaConfig, layer_idx=0):
        super().__init__()
        self.cfg = cfg
        self.n_q, self.n_kv, self.d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        std = cfg.initializer_range
        self.qkv_proj = _Linear(cfg.hidden_size, (self.n_q + 2 * self.n_kv) * self.d, std=std)
        self.o_proj = _Linear(self.n_q * self.d, cfg.hidden_size, std=std / math.sqrt(2 * cfg.num_hidden_layers))
        self.layer_idx = layer_idx
        self._register_load_state_dict_pre_hook(_fuse_hf_keys(("q_proj", "k_proj", "v_proj"), "qkv_proj"))

    sp_group = None  # Ulysses sequence-parallel group (parallel/ulysses.enable_sequence_parallel)
    fpdt = None  # FPDT settings (parallel/fpdt.enable_fpdt): chunked, optionally host-offloaded attention

    def forward(self, x, cos, sin, seq_len, cu_seqlens=None, pos_ids=None):
        T = x.shape[0]
        if self.fpdt is not None:
            from ..parallel.fpdt import fpdt_attention
            from .. import comm as dist
            f = self.fpdt
            assert cu_seqlens is None and not self.cfg.sliding_window, "FPDT: dense causal batches only"
            P = dist.get_world_size(f["group"]) if f["group"] is not None else 1
            nc = max(1, seq_len * P // f["chunk_size"])
            o = fpdt_attention(x, self.qkv_proj.weight, self.qkv_proj.bias, cos, sin, self.n_q, self.n_kv, self.d,
                               f["group"], T // seq_len, nc, offload=f["offload"])
            return self.o_proj(o)
        qkv = self.qkv_proj(x).view(T, self.n_q + 2 * self.n_kv, self.d)
        if self.sp_group is not None:
            from ..parallel.ulysses import local_heads, ulysses_out, ulysses_qkv
            from .. import comm as dist
            P = dist.get_world_size(self.sp_group)
            B = T // seq_len
            lq, lkv = local_heads(self.n_q, self.n_kv, self.sp_group)  # uneven heads / GQA with n_kv < sp
            full = ulysses_qkv(qkv, self.n_q, self.n_kv, self.sp_group, B)
            o = qkv_attention(full, lq, lkv, cos, sin, seq_len=seq_len * P, causal=True,
                              window=self.cfg.sliding_window)
            o = ulysses_out(o.view(B * seq_len * P, lq, self.d), self.sp_group, B, self.n_q, self.n_kv).reshape(T, -1)
            return self.o_proj(o)
        o = qkv_attention(qkv, self.n_q, self.n_kv, cos, sin, seq_len=seq_len, causal=True, cu_seqlens=cu_seqlens,
                          pos_ids=pos_ids, window=self.cfg.sliding_window)
        return self.o_proj(o)


class LlamaMLP(nn.Module):

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        std = cfg.initializer_range
        self.gate_up_proj = _Linear(cfg.hidden_size, 2 * cfg.intermediate_size, std=std)
        self.down_proj = _Linear(cfg.intermediate_size, cfg.hidden_size,
                                 std=std / math.sqrt(2 * cfg.num_hidden_layers))
        self.act = cfg.hidden_act
        self._register_load_state_dict_pre_hook(_fuse_hf_keys(("gate_proj", "up_proj"), "gate_up_proj"))

    fpdt_chunks = 0  # >1: sequence-chunked MLP with per-chunk recompute (parallel/fpdt.enable_fpdt)
    # long context: above ``chunk_min_tokens`` tokens the MLP runs in sequence chunks of ``chunk_rows`` rows, each
    # recomputed in backward (parallel/fpdt.fpdt_gated_ffn) -- at 512k tokens the gate|up output alone is 28 GiB and
    # its SwiGLU output + transpose another 28. Below the threshold the whole-sequence MLP is faster (no second
    # gate|up GEMM, NT-layout weight gradients; 128k: 8 % per step) and fits. 0: never
    chunk_rows = int(os.environ.get("HDS_MLP_CHUNK_ROWS", "65536"))
    chunk_min_tokens = int(os.environ.get("HDS_MLP_CHUNK_MIN_TOKENS", str(256 * 1024)))

    def forward(self, x):
        nc = self.fpdt_chunks
        if nc <= 1 and self.chunk_rows and x.shape[0] > max(self.chunk_rows, self.chunk_min_tokens):
            nc = -(-x.shape[0] // self.chunk_rows)
        if nc > 1:
            from ..parallel.fpdt import fpdt_gated_ffn
            return fpdt_gated_ffn(x, self.gate_up_proj.weight, self.down_proj.weight, nc, self.act)
        # ZeRO linears on both sides: the SwiGLU kernels also write the transposes the two weight gradients read
        # (runtime/zero/linear.py), instead of separate HBM transposes in the backward
        t = (torch.is_grad_enabled() and getattr(self.down_proj, "_hds_mel", False)
             and getattr(self.gate_up_proj, "_hds_mel", False))
        return self.down_proj(glu(self.gate_up_proj(x), self.act, transposed=t))


class LlamaDecoderLayer(nn.Module):

    def __init__(self, cfg: LlamaConfig, layer_idx=0):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg, layer_idx)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.mlp = LlamaMLP(cfg)

    def forward(self, h, residual, cos, sin, seq_len, cu_seqlens=None, pos_ids=None, summed=False):
        """h: output of the previous block (added to ``residual`` inside the fused norm).

        ``summed``: the block boundary is the summed residual stream s (``h`` = s, ``residual`` None) and the block
        returns ONE tensor, s + attn + mlp. A checkpointed block then saves one [tokens, hidden] input instead of
        two (h and residual), which halves what ckpt_offload spills and prefetches per block; the extra add is one
        elementwise pass."""
        if residual is None:
            x = self.input_layernorm(h)
            residual = h
        else:
            x, residual = self.input_layernorm(h, residual)
        a = self.self_attn(x, cos, sin, seq_len, cu_seqlens, pos_ids)
        x, residual = self.post_attention_layernorm(a, residual)
        if summed:
            return residual + self.mlp(x)
        return self.mlp(x), residual


class LlamaModel(nn.Module):

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed_tokens = _Embedding(cfg.vocab_size, cfg.hidden_size, std=cfg.initializer_range)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.gradient_checkpointing = False
        # block boundary = the summed residual stream (one saved tensor per checkpointed block, see
        # LlamaDecoderLayer.forward); set by the host activation cache's ckpt_offload policy, and used by plain
        # activation checkpointing
        self.summed_boundary = False

    def rope(self, device, max_pos):
        return rope_tables(max(max_pos, self.cfg.max_position_embeddings), self.cfg.head_dim, self.cfg.rope_theta,
                           self.cfg.rope_scaling, device=device)

    def forward(self, input_ids, cu_seqlens=None, pos_ids=None, layer_hook=None):
        """input_ids: [B, S] (or [T] + cu_seqlens). Returns final normed hidden [T, H]."""
        if input_ids.dim() == 2:
            B, S = input_ids.shape
            ids = input_ids.reshape(-1)
        else:
            ids, S = input_ids, input_ids.shape[0]
        h = self.embed_tokens(ids)
        sp = getattr(self, "_hds_sp_size", 1)
        cos, sin = self.rope(h.device, S * sp)
        if (getattr(self, "_domino_group", None) is not None and input_ids.dim() == 2 and B % 2 == 0
                and cu_seqlens is None and layer_hook is None and not self.gradient_checkpointing):
            from ..parallel.domino import domino_decoder_forward
            h, residual = domino_decoder_forward(self, h, cos, sin, S, B)
            h, _ = self.norm(h, residual)
            return h
        residual = None
        ckpt = self.gradient_checkpointing and self.training
        if (self.summed_boundary or ckpt) and layer_hook is None and torch.is_grad_enabled():
            for layer in self.layers:
                if ckpt:
                    h = _ckpt(layer, h, None, cos, sin, S, cu_seqlens, pos_ids, True)
                else:
                    h = layer(h, None, cos, sin, S, cu_seqlens, pos_ids, True)
            return self.norm(h)
        for i, layer in enumerate(self.layers):
            if layer_hook is not None:
                layer_hook(i, h, residual)
            if ckpt:
                h, residual = _ckpt(layer, h, residual, cos, sin, S, cu_seqlens, pos_ids)
            else:
                h, residual = layer(h, residual, cos, sin, S, cu_seqlens, pos_ids)
        h, _ = self.norm(h, residual)
        return h


class LlamaForCausalLM(nn.Module):

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        self.model = LlamaModel(cfg)
        self.lm_head = _Linear(cfg.hidden_size, cfg.vocab_size, std=cfg.initializer_range)
        if cfg.tie_word_embeddings:
            self.lm_head.weight = self.model.embed_tokens.weight
        # LM-head + CE row chunk: each chunk costs one fp32 read-modify-write of the [V, H] weight-gradient
        # accumulator, so fewer, larger chunks trade ~V*2 bytes of logits per extra row for less HBM traffic
        self.ce_chunk_rows = int(os.environ.get("HDS_CE_CHUNK_ROWS", "4096"))

    def gradient_checkpointing_enable(self):
        self.model.gradient_checkpointing = True

    def forward(self, input_ids, labels=None, cu_seqlens=None, pos_ids=None, return_hidden=False, targets=None):
        """``labels``: HF convention (shifted inside). ``targets``: already next-token aligned with
        ``input_ids`` (required with sequence parallelism, where a rank holds a slice of each sequence)."""
        h = self.model(input_ids, cu_seqlens=cu_seqlens, pos_ids=pos_ids)
        if return_hidden:
            return h
        if targets is not None:
            return fused_linear_cross_entropy(h, self.lm_head.weight, targets.reshape(-1),
                                              chunk_rows=self.ce_chunk_rows)
        if labels is None:
            return F.linear(h, self.lm_head.weight)
        lab = labels.reshape(-1) if labels.dim() > 1 else labels
        # next-token targets: shift left within each sequence, last position ignored
        if labels.dim() == 2:
            tgt = torch.full_like(labels, -100)
            tgt[:, :-1] = labels[:, 1:]
            tgt = tgt.reshape(-1)
        elif cu_seqlens is not None:
            tgt = torch.full_like(lab, -100)
            tgt[:-1] = lab[1:]
            tgt[(cu_seqlens[1:] - 1).long()] = -100
        else:
            tgt = torch.full_like(lab, -100)
            tgt[:-1] = lab[1:]
        return fused_linear_cross_entropy(h, self.lm_head.weight, tgt, chunk_rows=self.ce_chunk_rows)


def convert_hf_state_dict(sd, cfg: LlamaConfig):
    """HF LlamaForCausalLM state_dict -> this model's fused layout."""
    out = {}
    for k, v in sd.items():
        if ".q_proj." in k or ".k_proj." in k or ".v_proj." in k or ".gate_proj." in k or ".up_proj." in k:
            continue
        if "rotary_emb" in k:
            continue
        out[k] = v
    for i in range(cfg.num_hidden_layers):
        p = f"model.layers.{i}."
        out[p + "self_attn.qkv_proj.weight"] = torch.cat(
            [sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"], sd[p + "self_attn.v_proj.weight"]], 0)
        out[p + "mlp.gate_up_proj.weight"] = torch.cat([sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"]], 0)
    return out


def to_hf_state_dict(sd, cfg: LlamaConfig):
    """This model's fused layout -> HF LlamaForCausalLM names (q/k/v_proj, gate/up_proj). Inverse of
    :func:`convert_hf_state_dict`; use it to export checkpoints for HF / reference tooling."""
    out = {}
    qd, kd = cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim
    for k, v in sd.items():
        if k.endswith("self_attn.qkv_proj.weight"):
            base = k[:-len("qkv_proj.weight")]
            q, kk, vv = v.split([qd, kd, kd], 0)
            out[base + "q_proj.weight"], out[base + "k_proj.weight"], out[base + "v_proj.weight"] = q, kk, vv
        elif k.endswith("mlp.gate_up_proj.weight"):
            base = k[:-len("gate_up_proj.weight")]
            g, u = v.chunk(2, 0)
            out[base + "gate_proj.weight"], out[base + "up_proj.weight"] = g, u
        else:
            out[k] = v
    return out


def build(preset="llama3-8b", **overrides):
    cfg = PRESETS[preset](**overrides)
    return LlamaForCausalLM(cfg)
