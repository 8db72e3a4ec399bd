"""Layer configs the inference-v2 module heuristics select implementations from
(reference inference/v2/modules/configs/*.py)."""
from dataclasses import dataclass
from typing import Optional

import torch


@dataclass
class DSSelfAttentionConfig:
    n_heads_q: int
    n_heads_kv: int
    head_size: int
    max_sequences: int = 512
    scale_factor: float = 1.0
    positional_embedding_type: str = "rotate_half"  # or "none"
    rotary_dim: int = 0
    sliding_window: int = 0
    input_dtype: torch.dtype = torch.bfloat16


@dataclass
class DSLinearConfig:
    in_channels: int
    out_channels: int
    activation: str = "identity"  # identity | gelu | gelu_tanh | relu | silu | *_glu (gated, fused on [gate; up])
    input_dtype: torch.dtype = torch.bfloat16
    output_dtype: torch.dtype = torch.bfloat16
    quantization_mode: Optional[str] = None  # None | "wf6af16" | "int8" | "int4"
    group_size: int = 128


@dataclass
class DSMoEConfig:
    model_dim: int
    intermediate_features: int
    n_experts: int
    top_k: int = 2
    activation: str = "silu_glu"
    normalize_scores: bool = True
    input_dtype: torch.dtype = torch.bfloat16


@dataclass
class DSNormConfig:
    channels: int
    type: str = "rms"  # rms | layer
    eps: float = 1e-5
    residual_dtype: torch.dtype = torch.bfloat16
    input_dtype: torch.dtype = torch.bfloat16


@dataclass
class DSEmbeddingsConfig:
    residual_dtype: torch.dtype = torch.bfloat16
    embedding_dim: int = 0
    positional_embedding: bool = False
    positional_offset: int = 0


@dataclass
class DSUnembedConfig:
    max_sequences: int = 512
    dtype: torch.dtype = torch.bfloat16
    model_dim: int = 0
    vocab_size: int = 0
    norm_type: Optional[str] = "rms"  # final norm fused in front of the vocab GEMM (None: none)
