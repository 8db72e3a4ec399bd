"""Group-wise quantization ops: INT8/INT4 (sym/asym), FP8 (e4m3/e5m2), fake-quant, dequant-reduce.

Reference parity: ops/quantizer (``ds_quantizer``, csrc/quantization pt_binding: ``quantize``,
``dequantize``, ``swizzle_quant``, ``quantized_reduction``, fake-quant) and ops/fp_quantizer
(``FP_Quantize.quantize/dequantize/selective_dequantize`` :43). GPU path: csrc/kernels/quant.hip; CPU
path: the same math in torch (used by the CPU tests and as the numerics reference).
"""
import torch

from . import native

_FP8_MAX = {"e4m3": 448.0, "e5m2": 57344.0}


def _groups(x, group_size):
    n = x.numel()
    if n % group_size:
        raise ValueError(f"numel {n} not divisible by group_size {group_size}")
    return n // group_size


# ----------------------------------------------------------------------------------------
# INT8 / INT4
# ----------------------------------------------------------------------------------------
def _ref_quant_int(x, group_size, bits, symmetric):
    g = x.float().reshape(-1, group_size)
    if symmetric:
        qmax = 2**(bits - 1) - 1
        scale = g.abs().amax(1) / qmax
        scale = torch.where(scale > 0, scale, torch.ones_like(scale))
        q = torch.clamp(torch.round(g / scale[:, None]), -qmax - 1, qmax).to(torch.int8)
        mins = None
    else:
        qr = 2**bits - 1
        lo, hi = g.amin(1), g.amax(1)
        scale = torch.where(hi > lo, (hi - lo) / qr, torch.ones_like(hi))
        q = torch.clamp(torch.round((g - lo[:, None]) / scale[:, None]), 0, qr).to(torch.uint8).to(torch.int16)
        q = q.to(torch.int8) if bits == 4 else q.to(torch.uint8).view(torch.int8)
        mins = lo
    if bits == 4:
        u = (q.to(torch.int16) & 0xF).to(torch.uint8).reshape(-1, 2)
        q = (u[:, 0] | (u[:, 1] << 4)).view(torch.int8)
    return q.reshape(-1), scale, mins


def _ref_dequant_int(q, scale, mins, group_size, bits, symmetric, dtype):
    if bits == 4:
        u = q.view(torch.uint8)
        lo_n = (u & 0xF).to(torch.int16)
        hi_n = (u >> 4).to(torch.int16)
        vals = torch.stack([lo_n, hi_n], 1).reshape(-1)
        if symmetric:
            vals = (vals ^ 8) - 8
    else:
        vals = q.to(torch.int16) if symmetric else q.view(torch.uint8).to(torch.int16)
    g = vals.float().reshape(-1, group_size) * scale[:, None]
    if not symmetric:
        g = g + mins[:, None]
    return g.reshape(-1).to(dtype)


def quantize(x, group_size=512, bits=8, symmetric=True):
    """Returns (q int8 [numel or numel/2], scales fp32 [groups], mins fp32 [groups] | None)."""
    assert bits in (4, 8)
    x = x.contiguous()
    ng = _groups(x, group_size)
    if native.use_native(x):
        q = torch.empty(x.numel() * bits // 8, dtype=torch.int8, device=x.device)
        scales = torch.empty(ng, dtype=torch.float32, device=x.device)
        mins = None if symmetric else torch.empty(ng, dtype=torch.float32, device=x.device)
        native.check(native.kernels().hds_quant_int(native.dt(x), x.data_ptr(), q.data_ptr(), scales.data_ptr(),
                                                    0 if mins is None else mins.data_ptr(), ng, group_size, bits,
                                                    int(symmetric), native.stream()), "quant_int")
        return q, scales, mins
    return _ref_quant_int(x, group_size, bits, symmetric)


def dequantize(q, scales, mins=None, group_size=512, bits=8, symmetric=True, dtype=torch.bfloat16, out=None):
    ng = scales.numel()
    if native.use_native(q):
        y = out if out is not None else torch.empty(ng * group_size, dtype=dtype, device=q.device)
        native.check(native.kernels().hds_dequant_int(native.dt(y), q.data_ptr(), scales.data_ptr(),
                                                      0 if mins is None else mins.data_ptr(), y.data_ptr(), ng,
                                                      group_size, bits, int(symmetric), native.stream()),
                     "dequant_int")
        return y
    y = _ref_dequant_int(q, scales, mins, group_size, bits, symmetric, dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def fake_quantize(x, group_size=512, bits=8, symmetric=True):
    """Quantize-dequantize (QAT / MoQ), same dtype and shape as ``x``. 4/8-bit use the packed HIP kernels; other
    widths (MoQ walks 16 -> target bits one at a time) use the same group math in torch."""
    if bits not in (4, 8):
        g = x.float().reshape(-1, group_size)
        if symmetric:
            qmax = 2**(bits - 1) - 1
            sc = (g.abs().amax(1, keepdim=True) / qmax).clamp_min(1e-12)
            y = torch.clamp(torch.round(g / sc), -qmax - 1, qmax) * sc
        else:
            lo, hi = g.amin(1, keepdim=True), g.amax(1, keepdim=True)
            sc = ((hi - lo) / (2**bits - 1)).clamp_min(1e-12)
            y = torch.clamp(torch.round((g - lo) / sc), 0, 2**bits - 1) * sc + lo
        return y.reshape(x.shape).to(x.dtype)
    q, s, m = quantize(x, group_size, bits, symmetric)
    return dequantize(q, s, m, group_size, bits, symmetric, x.dtype).view_as(x)


def dequant_reduce(q, scales, world, n, group_size=512, bits=8, out=None, accumulate=False, dtype=torch.float32):
    """qgZ: ``out[i] (+)= sum_r dequant(q[r][i])`` for symmetric chunks q [world, n] (int4: n/2 bytes)."""
    if native.use_native(q):
        y = out if out is not None else torch.empty(n, dtype=dtype, device=q.device)
        native.check(native.kernels().hds_dequant_reduce(native.dt(y), q.data_ptr(), scales.data_ptr(), y.data_ptr(),
                                                         world, n, group_size, bits, int(accumulate),
                                                         native.stream()), "dequant_reduce")
        return y
    per = n * bits // 8
    tot = torch.zeros(n, dtype=torch.float32, device=q.device)
    ng = n // group_size
    for r in range(world):
        tot += _ref_dequant_int(q.reshape(-1)[r * per:(r + 1) * per], scales.reshape(-1)[r * ng:(r + 1) * ng], None,
                                group_size, bits, True, torch.float32)
    if out is not None:
        if accumulate:
            out.add_(tot.to(out.dtype))
        else:
            out.copy_(tot)
        return out
    return tot.to(dtype)


# ----------------------------------------------------------------------------------------
# FP8
# ----------------------------------------------------------------------------------------
def _fp8_dtype(fmt):
    return torch.float8_e4m3fn if fmt == "e4m3" else torch.float8_e5m2


def quantize_fp8(x, group_size=512, fmt="e4m3"):
    """Returns (q uint8 [numel] in OCP ``fmt``, scales fp32 [groups])."""
    x = x.contiguous()
    ng = _groups(x, group_size)
    if native.use_native(x):
        q = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
        scales = torch.empty(ng, dtype=torch.float32, device=x.device)
        native.check(native.kernels().hds_quant_fp8(native.dt(x), x.data_ptr(), q.data_ptr(), scales.data_ptr(), ng,
                                                    group_size, int(fmt == "e5m2"), native.stream()), "quant_fp8")
        return q, scales
    g = x.float().reshape(-1, group_size)
    scale = g.abs().amax(1) / _FP8_MAX[fmt]
    scale = torch.where(scale > 0, scale, torch.ones_like(scale))
    q = (g / scale[:, None]).clamp(-_FP8_MAX[fmt], _FP8_MAX[fmt]).to(_fp8_dtype(fmt)).view(torch.uint8)
    return q.reshape(-1), scale


def dequantize_fp8(q, scales, group_size=512, fmt="e4m3", dtype=torch.bfloat16, out=None):
    ng = scales.numel()
    if native.use_native(q):
        y = out if out is not None else torch.empty(ng * group_size, dtype=dtype, device=q.device)
        native.check(native.kernels().hds_dequant_fp8(native.dt(y), q.data_ptr(), scales.data_ptr(), y.data_ptr(), ng,
                                                      group_size, int(fmt == "e5m2"), native.stream()), "dequant_fp8")
        return y
    y = (q.view(_fp8_dtype(fmt)).float().reshape(-1, group_size) * scales[:, None]).reshape(-1).to(dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


class FP_Quantize:
    """Reference ops/fp_quantizer/quantize.py:43 API (q_bits 8 -> FP8; mantissa 3 -> e4m3, 2 -> e5m2)."""

    def __init__(self, group_size=512):
        self.group_size = group_size
        self.orig_dtype = None
        self.orig_shape = None
        self.scale = None
        self.fmt = "e4m3"

    def quantize(self, input, q_bits=8, q_mantisa_bits=3, stochastic_mode=False, return_meta_tensor=False):
        assert q_bits == 8, "only 8-bit FP formats are supported on gfx950 here (FP6/FP12: not implemented)"
        self.fmt = "e4m3" if q_mantisa_bits == 3 else "e5m2"
        self.orig_dtype, self.orig_shape = input.dtype, input.shape
        q, s = quantize_fp8(input.reshape(-1), self.group_size, self.fmt)
        self.scale = s
        return (q, s) if return_meta_tensor else q

    def dequantize(self, input_q, fp_out=None, q_bits=8, q_mantisa_bits=3, scale=None):
        fmt = "e4m3" if q_mantisa_bits == 3 else "e5m2"
        s = scale if scale is not None else self.scale
        y = dequantize_fp8(input_q.reshape(-1), s, self.group_size, fmt, self.orig_dtype or torch.bfloat16)
        y = y.view(self.orig_shape) if self.orig_shape is not None and y.numel() == _numel(self.orig_shape) else y
        if fp_out is not None:
            fp_out.copy_(y.view_as(fp_out))
            return fp_out
        return y

    def selective_dequantize(self, input_q, indexes, fp_out=None, q_bits=8, q_mantisa_bits=3, scale=None):
        """Dequantize only rows ``indexes`` of a [rows, cols] quantized matrix (cols multiple of group_size)."""
        fmt = "e4m3" if q_mantisa_bits == 3 else "e5m2"
        s = scale if scale is not None else self.scale
        rows = self.orig_shape[0] if (input_q.dim() == 1 and self.orig_shape is not None) else input_q.shape[0]
        qr = input_q.reshape(rows, -1)[indexes]
        sr = s.reshape(rows, -1)[indexes]
        y = dequantize_fp8(qr.reshape(-1), sr.reshape(-1), self.group_size, fmt, self.orig_dtype or torch.bfloat16)
        y = y.view(len(indexes), -1)
        if fp_out is not None:
            fp_out.copy_(y.view_as(fp_out))
            return fp_out
        return y


def _numel(shape):
    n = 1
    for d in shape:
        n *= d
    return n


class Quantizer:
    """Reference ops/quantizer ``ds_quantizer`` entry: symmetric/asymmetric fake quantization of a tensor."""

    def __call__(self, x, groups=1, bits=8, sr=False, asym=False):
        gs = x.numel() // groups
        return fake_quantize(x.reshape(-1), gs, bits, not asym).view_as(x)


def ds_quantizer(x, groups=1, bits=8, sr=False, asym=False):
    return Quantizer()(x, groups, bits, sr, asym)
