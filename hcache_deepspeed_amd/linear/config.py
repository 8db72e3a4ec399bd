"""LoRA / quantization configs for OptimizedLinear (reference linear/config.py)."""
from dataclasses import dataclass, field
from typing import List

import torch


@dataclass
class LoRAConfig:
    lora_r: int = 64
    lora_alpha: float = 16.0
    base_weight_sharding: int = 1
    offload: bool = False
    offload_ratio: float = 0.0
    delay_lora_init: bool = False
    target_mods: List[str] = field(
        default_factory=lambda: ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"])


@dataclass
class QuantizationConfig:
    q_bits: int = 8
    mantissa_bits: int = 3
    group_size: int = 512
    q_dtype: torch.dtype = torch.uint8
    # MI355X: 8-bit e4m3 weights of 2-D linears also keep an MX-FP8 copy (e8m0 scale per 32 elements) and run
    # prefill/training-sized inputs on the block-scaled FP8 matrix cores, with the activations MX-quantized on
    # the fly (ops/fp8_gemm.py). Opt-in: the default keeps the reference's weight-only path (dequantize + bf16 GEMM),
    # whose numerics do not depend on the token count.
    mx_fp8: bool = False
