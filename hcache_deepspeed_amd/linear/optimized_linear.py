"""OptimizedLinear: LoRA adapters over a frozen base weight that is sharded across data-parallel ranks and/or
stored in FP8.

Reference parity: linear/optimized_linear.py (``OptimizedLinear.__new__`` :37 dispatching to ``nn.Linear`` /
``QuantizedLinear`` / ``LoRAOptimizedLinear`` :76; ``init_lora`` :125, ``full_weight`` :183 all-gathering the
base shards, ``forward`` :206: base(x) + (alpha/r) * B(A(x))). MI355X: the frozen base shard is the only copy
in HBM (1/base_weight_sharding of the weight), gathered with ONE all-gather per forward; FP8 base weights use
the gfx950 e4m3 conversion kernels; ``fuse_lora_weight``/``unfuse_lora_weight`` serve the hybrid engine.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist
from .config import LoRAConfig, QuantizationConfig
from .quantization import QuantizedLinear, QuantizedParameter, _mx_eligible, mx_linear


class OptimizedLinear(nn.Module):

    def __new__(cls, input_dim, output_dim, bias=False, lora_config=None, quantization_config=None, device=None,
                dtype=torch.bfloat16, linear_cls=nn.Linear):
        if lora_config is None and quantization_config is None:
            return linear_cls(input_dim, output_dim, bias=bias, dtype=dtype, device=device)
        if lora_config is None:
            return QuantizedLinear(input_dim, output_dim, bias=bias, quantization_config=quantization_config,
                                   dtype=dtype)
        return LoRAOptimizedLinear(input_dim, output_dim, bias=bias, lora_config=lora_config,
                                   quantization_config=quantization_config, dtype=dtype, device=device)


class LoRAOptimizedLinear(nn.Module):

    def __init__(self, input_dim, output_dim, bias=False, lora_config=None, quantization_config=None, device=None,
                 dtype=torch.bfloat16):
        super().__init__()
        assert not bias, "bias=True is not supported by LoRAOptimizedLinear"
        self.input_dim, self.output_dim = input_dim, output_dim
        self.lora_config = lora_config or LoRAConfig()
        self.quantization_config = quantization_config
        self.dtype = dtype
        self.zero_shards = self.lora_config.base_weight_sharding
        self.sharded_weight_size = int(math.ceil(input_dim * output_dim / self.zero_shards))
        self.fused = False
        w = torch.empty(output_dim, input_dim, dtype=dtype, device=device)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        flat = torch.zeros(self.sharded_weight_size * self.zero_shards, dtype=dtype, device=device)
        flat[:w.numel()] = w.reshape(-1)
        rank = dist.get_rank() if (self.zero_shards > 1 and dist.is_initialized()) else 0
        shard = flat[rank * self.sharded_weight_size:(rank + 1) * self.sharded_weight_size].clone()
        if quantization_config is not None:
            self.weight = QuantizedParameter(shard, quantization_config=quantization_config, dtype=dtype)
            if self.zero_shards == 1 and _mx_eligible(self.weight.quantization_config, output_dim, input_dim):
                self.weight.enable_mx((output_dim, input_dim))
        else:
            self.weight = nn.Parameter(shard, requires_grad=False)
        self.weight.ds_optim_param = False
        self.lora_scaling_factor = self.lora_config.lora_alpha / self.lora_config.lora_r
        self.lora_weight_1 = nn.Linear(input_dim, self.lora_config.lora_r, bias=False, dtype=dtype, device=device)
        self.lora_weight_2 = nn.Linear(self.lora_config.lora_r, output_dim, bias=False, dtype=dtype, device=device)
        if not self.lora_config.delay_lora_init:
            self.init_lora()

    def init_lora(self):
        nn.init.kaiming_uniform_(self.lora_weight_1.weight, a=math.sqrt(5))
        nn.init.zeros_(self.lora_weight_2.weight)  # adapter starts as identity (B = 0)

    def disable(self):
        self.lora_weight_1.weight.requires_grad_(False)
        self.lora_weight_2.weight.requires_grad_(False)

    def _shard(self):
        return self.weight.dequantized().reshape(-1) if isinstance(self.weight, QuantizedParameter) else self.weight

    def full_weight(self):
        shard = self._shard()
        if self.zero_shards > 1 and dist.is_initialized() and dist.get_world_size() > 1:
            full = torch.empty(self.sharded_weight_size * self.zero_shards, dtype=shard.dtype, device=shard.device)
            dist.all_gather_into_tensor(full, shard.contiguous())
        else:
            full = shard
        return full[:self.input_dim * self.output_dim].view(self.output_dim, self.input_dim)

    @torch.no_grad()
    def fuse_lora_weight(self):
        """Hybrid-engine generation: fold B.A into the base weight (single-shard weights only)."""
        if self.fused or self.zero_shards > 1 or isinstance(self.weight, QuantizedParameter):
            return
        delta = self.lora_scaling_factor * (self.lora_weight_2.weight @ self.lora_weight_1.weight)
        self.weight.data.add_(delta.reshape(-1).to(self.weight.dtype))
        self.fused = True

    @torch.no_grad()
    def unfuse_lora_weight(self):
        if not self.fused:
            return
        delta = self.lora_scaling_factor * (self.lora_weight_2.weight @ self.lora_weight_1.weight)
        self.weight.data.sub_(delta.reshape(-1).to(self.weight.dtype))
        self.fused = False

    def forward(self, x):
        if isinstance(self.weight, QuantizedParameter) and self.weight.mx_ok() and not self.fused:
            base = mx_linear(x, self.weight)
        else:
            base = F.linear(x, self.full_weight().to(x.dtype))
        if self.fused:
            return base
        return base + self.lora_scaling_factor * self.lora_weight_2(self.lora_weight_1(x))
