"""FP8-quantized frozen weights (reference linear/quantization.py ``QuantizedParameter`` :18 / ``QuantizedLinear``
:129). The weight is stored as OCP e4m3 (or e5m2) bytes + fp32 group scales produced by the gfx950 conversion
kernels (ops/quantizer.quantize_fp8) and dequantized to the compute dtype for each forward."""
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

    def _ensure_quantized(self, tensor):
        if tensor.numel() == 0:
            self.q_data, self.q_scales = tensor, None
            return
        gs = self.quantization_config.group_size
        flat = tensor.detach().reshape(-1)
        if flat.numel() % gs:
            gs = flat.numel()
        self.group_size = gs
        self.q_data, self.q_scales = Q.quantize_fp8(flat.contiguous(), gs, self.fmt)

    def dequantized(self):
        return Q.dequantize_fp8(self.q_data, self.q_scales, self.group_size, self.fmt,
                                self.orig_dtype).view(self.orig_shape)

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
        return F.linear(x, self.weight.dequantized().to(x.dtype), self.bias)
