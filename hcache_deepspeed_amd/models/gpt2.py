"""GPT-2 (learned positions, pre-LayerNorm, GELU MLP, tied embeddings) on this framework's fused ops.

BASELINE config "GPT-2-small ZeRO-1 on cpu_accelerator + gloo world_size=2" (plumbing check) and the
reference's BERT/GPT-style test models (tests/unit/simple_model.py, module_inject containers/gpt2.py).
LayerNorm uses the wave64 norm kernel (fused residual add), the MLP the bias+GELU kernel, attention the
HIP FlashAttention (causal) on GPU; every op has a torch reference path so the model also runs on CPU.
"""
import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activations import bias_act
from ..ops.attention import flash_attn, native_supported
from ..ops.cross_entropy import fused_linear_cross_entropy
from ..ops.norm import LayerNorm
from ..runtime.activation_checkpointing.checkpointing import checkpoint as _ckpt


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_epsilon: float = 1e-5
    initializer_range: float = 0.02
    model_type: str = "gpt2"

    @property
    def head_dim(self):
        return self.n_embd // self.n_head

    def flops_per_token(self, seq_len):
        n = 12 * self.n_layer * self.n_embd**2
        return 6 * n + 6 * self.n_layer * seq_len * self.n_embd + 6 * self.n_embd * self.vocab_size


def gpt2_small(**kw):
    return GPT2Config(**kw)


def gpt2_medium(**kw):
    return GPT2Config(**dict(dict(n_embd=1024, n_layer=24, n_head=16), **kw))


def gpt2_tiny(**kw):
    return GPT2Config(**dict(dict(vocab_size=256, n_positions=128, n_embd=64, n_layer=2, n_head=4), **kw))


class GPT2Block(nn.Module):

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        H = cfg.n_embd
        self.n_head = cfg.n_head
        self.ln_1 = LayerNorm(H, cfg.layer_norm_epsilon)
        self.c_attn = nn.Linear(H, 3 * H)
        self.c_proj = nn.Linear(H, H)
        self.ln_2 = LayerNorm(H, cfg.layer_norm_epsilon)
        self.c_fc = nn.Linear(H, 4 * H)
        self.c_proj2 = nn.Linear(4 * H, H)
        std = cfg.initializer_range
        for lin in (self.c_attn, self.c_fc):
            nn.init.normal_(lin.weight, std=std)
            nn.init.zeros_(lin.bias)
        for lin in (self.c_proj, self.c_proj2):
            nn.init.normal_(lin.weight, std=std / math.sqrt(2 * cfg.n_layer))
            nn.init.zeros_(lin.bias)

    def _attn(self, x, B, S):
        H = x.shape[-1]
        D = H // self.n_head
        qkv = self.c_attn(x).view(B, S, 3, self.n_head, D)
        q, k, v = qkv.unbind(2)
        if native_supported(x.view(-1, self.n_head, D)):
            o = flash_attn(q.contiguous(), k.contiguous(), v.contiguous(), causal=True)
        else:
            o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                               is_causal=True).transpose(1, 2)
        return self.c_proj(o.reshape(B * S, H))

    def forward(self, h, residual, B, S):
        if residual is None:
            x = self.ln_1(h)
            residual = h
        else:
            x, residual = self.ln_1(h, residual)
        a = self._attn(x, B, S)
        x, residual = self.ln_2(a, residual)
        y = bias_act(F.linear(x, self.c_fc.weight), self.c_fc.bias, "gelu_tanh")
        return self.c_proj2(y), residual


class GPT2LMHeadModel(nn.Module):

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.config = cfg
        self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        nn.init.normal_(self.wte.weight, std=cfg.initializer_range)
        nn.init.normal_(self.wpe.weight, std=0.01)
        self.h = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(cfg.n_embd, cfg.layer_norm_epsilon)
        self.gradient_checkpointing = False

    def gradient_checkpointing_enable(self):
        self.gradient_checkpointing = True

    def forward(self, input_ids, labels=None):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        h = (self.wte(input_ids) + self.wpe(pos)[None]).reshape(B * S, -1)
        residual = None
        for blk in self.h:
            if self.gradient_checkpointing and self.training:
                h, residual = _ckpt(blk, h, residual, B, S)
            else:
                h, residual = blk(h, residual, B, S)
        h, _ = self.ln_f(h, residual)
        if labels is None:
            return F.linear(h, self.wte.weight).view(B, S, -1)
        tgt = torch.full_like(labels, -100)
        tgt[:, :-1] = labels[:, 1:]
        return fused_linear_cross_entropy(h, self.wte.weight, tgt.reshape(-1))


def convert_hf_state_dict(sd):
    """HF GPT2LMHeadModel state_dict (Conv1D weights [in, out]) -> this model's names/layout."""
    out = {}
    for k, v in sd.items():
        k2 = k[len("transformer."):] if k.startswith("transformer.") else k
        if k2.startswith("lm_head") or k2.endswith(".attn.bias") or k2.endswith(".attn.masked_bias"):
            continue
        k2 = k2.replace(".attn.c_attn.", ".c_attn.").replace(".attn.c_proj.", ".c_proj.")
        k2 = k2.replace(".mlp.c_fc.", ".c_fc.").replace(".mlp.c_proj.", ".c_proj2.")
        if k2.endswith(".weight") and any(s in k2 for s in (".c_attn.", ".c_proj.", ".c_fc.", ".c_proj2.")):
            v = v.t().contiguous()
        out[k2] = v
    return out
