"""Mixtral-style sparse MoE causal LM (Llama attention + top-k SwiGLU experts with expert parallelism).

BASELINE config "Mixtral 8x7B ZeRO-3 + expert-parallel all-to-all over xGMI". Reference parity: the HF
Mixtral model trained through deepspeed.initialize with moe/layer.MoE, and inference/v2
model_implementations/mixtral (serving).
"""
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.cross_entropy import fused_linear_cross_entropy
from ..ops.norm import RMSNorm
from ..parallel.moe import MoE
from ..runtime.activation_checkpointing.checkpointing import checkpoint as _ckpt
from .llama import LlamaAttention, LlamaConfig, _Embedding, _Linear


@dataclass
class MixtralConfig(LlamaConfig):
    num_local_experts: int = 8
    num_experts_per_tok: int = 2
    router_aux_loss_coef: float = 0.02
    capacity_factor: float = 1.25
    drop_tokens: bool = True
    ep_size: int = 1
    model_type: str = "mixtral"

    def num_params(self, include_embedding=True):
        H, I, L, V = self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size
        D, Hq, Hkv, E = self.head_dim, self.num_attention_heads, self.num_key_value_heads, self.num_local_experts
        per_layer = H * (Hq + 2 * Hkv) * D + Hq * D * H + E * 3 * H * I + H * E + 2 * H
        n = L * per_layer + H
        if include_embedding:
            n += V * H * 2
        return n

    def flops_per_token(self, seq_len):
        """Training FLOPs/token with only the top-k experts counted (+ router)."""
        return 6 * (self.active_params() + self.num_hidden_layers * self.hidden_size * self.num_local_experts) + \
            6 * self.vocab_size * self.hidden_size + 12 * self.num_hidden_layers * self.hidden_size * seq_len

    def active_params(self):
        H, I, L = self.hidden_size, self.intermediate_size, self.num_hidden_layers
        D, Hq, Hkv, k = self.head_dim, self.num_attention_heads, self.num_key_value_heads, self.num_experts_per_tok
        return L * (H * (Hq + 2 * Hkv) * D + Hq * D * H + k * 3 * H * I)


def mixtral_8x7b(**kw):
    d = dict(vocab_size=32000, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
             num_attention_heads=32, num_key_value_heads=8, rope_theta=1e6, max_position_embeddings=32768)
    d.update(kw)
    return MixtralConfig(**d)


def tiny_moe(**kw):
    d = dict(vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2, num_attention_heads=2,
             num_key_value_heads=1, head_dim=128, num_local_experts=4, num_experts_per_tok=2)
    d.update(kw)
    return MixtralConfig(**d)


class MixtralDecoderLayer(nn.Module):

    def __init__(self, cfg: MixtralConfig, layer_idx=0):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg, layer_idx)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.block_sparse_moe = MoE(cfg.hidden_size, None, cfg.num_local_experts, cfg.ep_size,
                                    k=cfg.num_experts_per_tok, capacity_factor=cfg.capacity_factor,
                                    eval_capacity_factor=cfg.capacity_factor, drop_tokens=cfg.drop_tokens,
                                    use_rts=False, expert_intermediate_size=cfg.intermediate_size)

    def forward(self, h, residual, cos, sin, seq_len, cu_seqlens=None, pos_ids=None):
        if residual is None:
            x = self.input_layernorm(h)
            residual = h
        else:
            x, residual = self.input_layernorm(h, residual)
        a = self.self_attn(x, cos, sin, seq_len, cu_seqlens, pos_ids)
        x, residual = self.post_attention_layernorm(a, residual)
        out, l_aux, _ = self.block_sparse_moe(x)
        self.l_aux = l_aux
        return out, residual


class MixtralForCausalLM(nn.Module):

    def __init__(self, cfg: MixtralConfig):
        super().__init__()
        self.config = cfg
        self.embed_tokens = _Embedding(cfg.vocab_size, cfg.hidden_size, std=cfg.initializer_range)
        self.layers = nn.ModuleList([MixtralDecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.lm_head = _Linear(cfg.hidden_size, cfg.vocab_size, std=cfg.initializer_range)
        self.gradient_checkpointing = False

    def forward(self, input_ids, labels=None, targets=None):
        from ..ops.rope import rope_tables
        B, S = input_ids.shape
        h = self.embed_tokens(input_ids.reshape(-1))
        cos, sin = rope_tables(max(S, self.config.max_position_embeddings), self.config.head_dim,
                               self.config.rope_theta, self.config.rope_scaling, device=h.device)
        residual = None
        aux = 0.0
        for layer in self.layers:
            if self.gradient_checkpointing and self.training:
                h, residual = _ckpt(layer, h, residual, cos, sin, S)
            else:
                h, residual = layer(h, residual, cos, sin, S)
            aux = aux + layer.l_aux
        h, _ = self.norm(h, residual)
        if labels is None and targets is None:
            return F.linear(h, self.lm_head.weight)
        if targets is None:
            targets = torch.full_like(labels, -100)
            targets[:, :-1] = labels[:, 1:]
        loss = fused_linear_cross_entropy(h, self.lm_head.weight, targets.reshape(-1))
        return loss + self.config.router_aux_loss_coef * aux / len(self.layers)
