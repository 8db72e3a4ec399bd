"""Quantized frozen weights (reference linear/quantization.py ``QuantizedParameter`` :18 / ``QuantizedLinear``
:129). ``q_bits=8``: OCP e4m3 (or e5m2) bytes + fp32 group scales from the gfx950 conversion instructions
(ops/quantizer.quantize_fp8). ``q_bits=6`` / ``12``: packed FP6 (e3m2 / e2m3) or FP12 minifloats (csrc/kernels/
fpq.hip). The weight is dequantized to the compute dtype for each forward; FP6 linears with decode-sized inputs
skip that and run the fused 6-bit GEMV (ops/quantizer.fp6_linear)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import quantizer as Q
from .config import QuantizationConfig


class QuantizedParameter(nn.Parameter):

    def __new__(cls, data=None, requires_grad=False, quantization_config=None, dtype=None):
        if data is None:
            data = torch.empty(0)
        self = torch.Tensor._make_subclass(cls, torch.empty(0, dtype=torch.uint8, device=data.device), False)
        self.quantization_config = quantization_config or QuantizationConfig()
        self.orig_dtype = dtype or (data.dtype if data.is_floating_point() else torch.bfloat16)
        self.orig_shape = tuple(data.shape)
        self._ensure_quantized(data)
        return self

    @property
    def fmt(self):
        return "e4m3" if self.quantization_config.mantissa_bits == 3 else "e5m2"

    @property
    def q_bits(self):
        return self.quantization_config.q_bits

    def _ensure_quantized(self, tensor):
        if tensor.numel() == 0:
            self.q_data, self.q_scales = tensor, None
            return
        gs = self.quantization_config.group_size
        flat = tensor.detach().reshape(-1)
        if flat.numel() % gs:
            gs = flat.numel()
        self.group_size = gs
        if self.q_bits == 8:
            self.q_data, self.q_scales = Q.quantize_fp8(flat.contiguous(), gs, self.fmt)
        else:
            self.q_data, self.q_scales = Q.quantize_minifloat(flat.contiguous(), gs, self.q_bits,
                                                              self.quantization_config.mantissa_bits)

    def dequantized(self):
        if self.q_bits == 8:
            return Q.dequantize_fp8(self.q_data, self.q_scales, self.group_size, self.fmt,
                                    self.orig_dtype).view(self.orig_shape)
        return Q.dequantize_minifloat(self.q_data, self.q_scales, self.group_size, self.q_bits,
                                      self.quantization_config.mantissa_bits, self.orig_dtype).view(self.orig_shape)

    def offload(self, revert=False):
        dev = "cuda" if revert and torch.cuda.is_available() else "cpu"
        self.q_data = self.q_data.to(dev)
        self.q_scales = self.q_scales.to(dev)

    def to(self, *args, **kwargs):
        dev = None
        for a in args:
            if isinstance(a, (str, torch.device)):
                dev = a
        dev = kwargs.get("device", dev)
        if dev is not None:
            self.q_data = self.q_data.to(dev)
            self.q_scales = self.q_scales.to(dev)
        return self

    def cuda(self, device=None, non_blocking=False):
        return self.to(device or "cuda")


class QuantizedLinear(nn.Linear):

    def __init__(self, input_dim, output_dim, bias=False, quantization_config=None, dtype=torch.bfloat16):
        super().__init__(input_dim, output_dim, bias=bias, dtype=dtype)
        self.weight = QuantizedParameter(self.weight.data, quantization_config=quantization_config, dtype=dtype)

    def forward(self, x):
        w = self.weight
        if w.q_bits == 6 and len(w.orig_shape) == 2 and w.orig_shape[1] % w.group_size == 0:
            y = Q.fp6_linear(x, w.q_data, w.q_scales, w.orig_shape[0], w.orig_shape[1], w.group_size,
                             w.quantization_config.mantissa_bits)
            return y + self.bias if self.bias is not None else y
        return F.linear(x, w.dequantized().to(x.dtype), self.bias)
