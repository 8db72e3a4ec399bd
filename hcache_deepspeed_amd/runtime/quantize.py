"""MoQ: mixture-of-quantization training (weights fake-quantized with a bit-width schedule).

Reference parity: runtime/quantize.py (``Quantizer`` :14: start/target bits, period doubling per bit drop,
optional eigenvalue-scaled periods, symmetric/asymmetric, fp16 mixing ratio). The per-step quantize uses the
HIP group-quantization kernel (ops/quantizer.fake_quantize) on GPU.
"""
import torch

from ..ops.quantizer import fake_quantize


class Quantizer:

    def __init__(self, q_groups=1, q_mixed_fp16=False, q_change_ratio=0.01, q_type=0, q_rounding=0,
                 q_verbose=False, q_eigenvalue=False, use_quantizer_kernel=True, layer_num=0):
        self.q_groups = q_groups
        self.q_mixed_fp16 = q_mixed_fp16
        self.q_change_ratio = q_change_ratio
        self.q_type = q_type  # 0 symmetric, 1 asymmetric
        self.q_rounding = q_rounding
        self.q_verbose = q_verbose
        self.q_eigenvalue = q_eigenvalue
        self.use_quantizer_kernel = use_quantizer_kernel
        self.layer_num = layer_num
        self.qsteps = 0
        self.quantize_real_ratio = 1.0

    def any_precision_switch(self):
        return False

    def step(self):
        self.qsteps += 1

    def update_fp16_ratio(self):
        if self.q_mixed_fp16:
            self.quantize_real_ratio = max(0.0, self.quantize_real_ratio - self.q_change_ratio)

    def compute_quantization(self, x, bits):
        n = x.numel()
        groups = self.q_groups if n % self.q_groups == 0 else 1
        gs = n // groups
        if gs % 8:
            return x
        q = fake_quantize(x.reshape(-1).contiguous(), gs, bits, self.q_type == 0).view_as(x)
        if self.q_mixed_fp16 and self.quantize_real_ratio > 0:
            return self.quantize_real_ratio * x + (1 - self.quantize_real_ratio) * q
        return q

    @torch.no_grad()
    def quantize(self, parameter_group, overflow, eigenvalue_enabled=False, block_eigenvalue=None):
        """``parameter_group``: list of lists of params; each param may carry ``start_bits``, ``target_bits``,
        ``q_period`` attributes (set by init_compression / the config)."""
        if overflow and not eigenvalue_enabled:
            return
        self.step()
        self.update_fp16_ratio()
        for group in parameter_group:
            for p in group:
                if p.dim() < 2 or not hasattr(p, "start_bits"):
                    continue
                period = p.q_period
                if block_eigenvalue and hasattr(p, "block_id") and p.block_id in block_eigenvalue:
                    period = int(period * (1 + block_eigenvalue[p.block_id][0]))
                if self.qsteps >= period and p.start_bits > p.target_bits:
                    p.start_bits -= 1
                    p.q_period = period * 2
                p.data.copy_(self.compute_quantization(p.data, p.start_bits))
