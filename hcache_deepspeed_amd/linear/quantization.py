"""Quantized frozen weights (reference linear/quantization.py ``QuantizedParameter`` :18 / ``QuantizedLinear``
:129). ``q_bits=8``: OCP e4m3 (or e5m2) bytes + fp32 group scales from the gfx950 conversion instructions
(ops/quantizer.quantize_fp8). ``q_bits=6`` / ``12``: packed FP6 (e3m2 / e2m3) or FP12 minifloats (csrc/kernels/
fpq.hip). The weight is dequantized to the compute dtype for each forward; FP6 linears with decode-sized inputs
skip that and run the fused 6-bit GEMV (ops/quantizer.fp6_linear).

With ``QuantizationConfig.mx_fp8`` (opt-in; default off = the reference's weight-only numerics) 8-bit e4m3 2-D weights
additionally hold an MX-FP8 copy derived from the quantized weight: inputs of >= 256 rows
then run on the block-scaled FP8 matrix cores (ops/fp8_gemm.py, 1.5-1.8x the bf16 GEMM), forward AND the input
gradient of the frozen weight (a transposed MX copy made on first use)."""
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
        if getattr(self, "mx_shape", None) is not None:  # re-quantized: the MX copy follows the new q_data
            self.enable_mx(self.mx_shape)

    def enable_mx(self, shape2d):
        """Keep an MX-FP8 copy (logical shape ``shape2d`` = [out, in]) derived from the quantized weight itself, so
        the two paths see the same weight values."""
        from ..ops.fp8_gemm import mx_quantize
        N, K = shape2d
        self.mx_shape = (N, K)
        self.mx_w = mx_quantize(self.dequantized().reshape(N, K).to(torch.bfloat16).contiguous())
        self.mx_wt = None  # [in, out] copy for the input gradient, built on first backward

    def mx_ok(self):
        cfg = self.quantization_config
        return getattr(self, "mx_w", None) is not None and getattr(cfg, "mx_fp8", False)

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
        if getattr(self, "mx_w", None) is not None:
            self.mx_w = tuple(t.to(dev) for t in self.mx_w)
            self.mx_wt = None

    def to(self, *args, **kwargs):
        dev = None
        for a in args:
            if isinstance(a, (str, torch.device)):
                dev = a
        dev = kwargs.get("device", dev)
        if dev is not None:
            self.q_data = self.q_data.to(dev)
            self.q_scales = self.q_scales.to(dev)
            if getattr(self, "mx_w", None) is not None:
                self.mx_w = tuple(t.to(dev) for t in self.mx_w)
                self.mx_wt = None
        return self

    def cuda(self, device=None, non_blocking=False):
        return self.to(device or "cuda")


def _mx_eligible(cfg, N, K):
    from ..ops.fp8_gemm import mx_supported
    return cfg.q_bits == 8 and cfg.mantissa_bits == 3 and getattr(cfg, "mx_fp8", False) and mx_supported(256, N, K)


class _MxLinearFn(torch.autograd.Function):
    """y = x . W^T on MX-FP8 (W frozen); dx = dy . W on the transposed MX copy."""

    @staticmethod
    def forward(ctx, x, w):
        from ..ops.fp8_gemm import fp8_linear
        ctx.w = w
        return fp8_linear(x, *w.mx_w)

    @staticmethod
    def backward(ctx, dy):
        from ..ops.fp8_gemm import fp8_linear, mx_dequantize, mx_quantize, mx_supported
        w = ctx.w
        N, K = w.mx_shape
        dy2 = dy.reshape(-1, N)
        if mx_supported(dy2.shape[0], K, N) and dy.is_cuda:
            if w.mx_wt is None:
                w.mx_wt = mx_quantize(mx_dequantize(*w.mx_w, dtype=torch.bfloat16).t().contiguous())
            dx = fp8_linear(dy2, *w.mx_wt)
        else:
            dx = dy2.float() @ mx_dequantize(*w.mx_w)
        return dx.to(dy.dtype).reshape(*dy.shape[:-1], K), None


def mx_linear(x, w):
    """F.linear(x, W) for a QuantizedParameter with an MX copy: FP8 matrix cores when the token count tiles,
    otherwise the dequantized weight."""
    from ..ops.fp8_gemm import mx_dequantize, mx_supported
    M = x.numel() // x.shape[-1]
    N, K = w.mx_shape
    if x.is_cuda and mx_supported(M, N, K):
        return _MxLinearFn.apply(x, w)
    return F.linear(x, mx_dequantize(*w.mx_w, dtype=x.dtype))


class QuantizedLinear(nn.Linear):

    def __init__(self, input_dim, output_dim, bias=False, quantization_config=None, dtype=torch.bfloat16):
        super().__init__(input_dim, output_dim, bias=bias, dtype=dtype)
        data = self.weight.data
        self.weight = QuantizedParameter(data, quantization_config=quantization_config, dtype=dtype)
        if _mx_eligible(self.weight.quantization_config, output_dim, input_dim):
            self.weight.enable_mx((output_dim, input_dim))

    def forward(self, x):
        w = self.weight
        if w.mx_ok():
            y = mx_linear(x, w)
            return y + self.bias if self.bias is not None else y
        if w.q_bits == 6 and len(w.orig_shape) == 2 and w.orig_shape[1] % w.group_size == 0:
            y = Q.fp6_linear(x, w.q_data, w.q_scales, w.orig_shape[0], w.orig_shape[1], w.group_size,
                             w.quantization_config.mantissa_bits)
            return y + self.bias if self.bias is not None else y
        return F.linear(x, w.dequantized().to(x.dtype), self.bias)
