"""Group-wise quantization ops: INT8/INT4 (sym/asym), FP8 (e4m3/e5m2), fake-quant, dequant-reduce.

Reference parity: ops/quantizer (``ds_quantizer``, csrc/quantization pt_binding: ``quantize``,
``dequantize``, ``swizzle_quant``, ``quantized_reduction``, fake-quant) and ops/fp_quantizer
(``FP_Quantize.quantize/dequantize/selective_dequantize`` :43). GPU path: csrc/kernels/quant.hip; CPU
path: the same math in torch (used by the CPU tests and as the numerics reference).
"""
import os

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


_INT_GEMV_MAX_M = min(8, int(os.environ.get("HDS_INT_GEMV_MAX_M", "2")))


# above 64 rows dequantize-once + hipBLASLt wins on most shapes (profiles/wmix_bench_r2.log)
_WMIX_MAX_M = int(os.environ.get("HDS_WMIX_MAX_M", "64"))


def _needs_grad(x):
    """The fused GEMV / mixed-input kernels have no backward: an input that needs a gradient (a LoRA base under
    training) takes the differentiable dequantize + GEMM path so dX still flows to earlier layers."""
    return torch.is_grad_enabled() and x.requires_grad


def wmix_eligible(x2, out_features, in_features, group_size):
    M = x2.shape[0]
    return (not _needs_grad(x2) and native.use_native(x2) and x2.dtype == torch.bfloat16 and 0 < M <= _WMIX_MAX_M
            and bool(native.kernels().hds_wmix_supported(M, out_features, in_features, group_size)))


def wmix_gemm(x2, q_weight, scales, out_features, in_features, group_size, fmt, ebits=3, bias=None):
    """Mixed-input MFMA GEMM (csrc/kernels/wmix_gemm.hip): bf16 [M, K] x packed weight [N, K] -> bf16 [M, N].
    fmt: "int8" | "int4" | "fp6". The packed weight is decoded in registers; it never exists in bf16 in HBM."""
    M = x2.shape[0]
    x2 = x2.contiguous()
    lib = native.kernels()
    splits = lib.hds_wmix_splits(M, out_features, in_features)
    y = torch.empty(M, out_features, dtype=torch.bfloat16, device=x2.device)
    ws = torch.empty(splits, M, out_features, dtype=torch.float32, device=x2.device) if splits > 1 else None
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    native.check(lib.hds_wmix_gemm(x2.data_ptr(), q_weight.data_ptr(), scales.data_ptr(), native.ptr(bias),
                                   y.data_ptr(), native.ptr(ws), M, out_features, in_features, group_size,
                                   {"int8": 0, "int4": 1, "fp6": 2}[fmt], int(ebits), native.stream()), "wmix_gemm")
    return y


def int_linear(x, q_weight, scales, out_features, in_features, group_size, bits=8, bias=None):
    """y = x @ dequant(W)^T for a symmetric group-quantized int8/int4 weight [out, in] (groups along ``in``).

    Decode-sized inputs (<= 2 rows by default, ``HDS_INT_GEMV_MAX_M``) run the fused HIP GEMV (csrc/kernels/quant.hip
    ``int_gemv_kernel``) that reads the packed weight straight from HBM (1.5-2.3x faster than the bf16 GEMM at one
    row, profiles/int_gemv_bench_r1.log); larger batches dequantize once to bf16 and use the matrix cores."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, in_features)
    M = x2.shape[0]
    if not _needs_grad(x2) and native.use_native(x2) and 0 < M <= _INT_GEMV_MAX_M and x2.dtype == torch.bfloat16 and in_features % 16 == 0 \
            and group_size % 16 == 0:
        x2 = x2.contiguous()
        y = torch.empty(M, out_features, dtype=torch.bfloat16, device=x.device)
        native.check(native.kernels().hds_int_gemv(x2.data_ptr(), q_weight.data_ptr(), scales.data_ptr(),
                                                   y.data_ptr(), M, out_features, in_features, group_size, bits,
                                                   native.stream()), "int_gemv")
        y = y.view(*lead, out_features)
        return y if bias is None else y + bias
    if wmix_eligible(x2, out_features, in_features, group_size):  # batched decode / chunked prefill: MFMA
        return wmix_gemm(x2, q_weight, scales, out_features, in_features, group_size, f"int{bits}",
                         bias=bias).view(*lead, out_features)
    w = dequantize(q_weight, scales, None, group_size, bits, True, x.dtype).view(out_features, in_features)
    return torch.nn.functional.linear(x, w, bias)


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
    """Reference ops/fp_quantizer/quantize.py:43 API: q_bits 8 (mantissa 3 -> e4m3, 2 -> e5m2), 6 (e3m2 / e2m3)
    or 12 (e4m7); ``stochastic_mode`` rounds stochastically (minifloat kernel)."""

    def __init__(self, group_size=512):
        self.group_size = group_size
        self.orig_dtype = None
        self.orig_shape = None
        self.scale = None
        self.fmt = "e4m3"

    def quantize(self, input, q_bits=8, q_mantisa_bits=3, stochastic_mode=False, return_meta_tensor=False):
        """FP8 (OCP e4m3 / e5m2 via the gfx950 cvt instructions) or FP6 / FP12 minifloats (fpq.hip)."""
        self.q_bits, self.q_mantisa_bits = q_bits, q_mantisa_bits
        self.orig_dtype, self.orig_shape = input.dtype, input.shape
        if q_bits == 8 and not stochastic_mode:
            self.fmt = "e4m3" if q_mantisa_bits == 3 else "e5m2"
            q, s = quantize_fp8(input.reshape(-1), self.group_size, self.fmt)
        else:
            q, s = quantize_minifloat(input.reshape(-1), self.group_size, q_bits, q_mantisa_bits,
                                      stochastic=stochastic_mode, seed=torch.randint(0, 2**31 - 1, (1, )).item())
            self.fmt = f"mini{q_bits}m{q_mantisa_bits}"
        self.scale = s
        return (q, s) if return_meta_tensor else q

    def _deq(self, q, s, q_bits, q_mantisa_bits):
        if q_bits == 8 and not getattr(self, "fmt", "e4m3").startswith("mini"):
            return dequantize_fp8(q, s, self.group_size, "e4m3" if q_mantisa_bits == 3 else "e5m2",
                                  self.orig_dtype or torch.bfloat16)
        return dequantize_minifloat(q, s, self.group_size, q_bits, q_mantisa_bits, self.orig_dtype or torch.bfloat16)

    def dequantize(self, input_q, fp_out=None, q_bits=8, q_mantisa_bits=3, scale=None):
        s = scale if scale is not None else self.scale
        y = self._deq(input_q.reshape(-1), s, q_bits, q_mantisa_bits)
        y = y.view(self.orig_shape) if self.orig_shape is not None and y.numel() == _numel(self.orig_shape) else y
        if fp_out is not None:
            fp_out.copy_(y.view_as(fp_out))
            return fp_out
        return y

    def selective_dequantize(self, input_q, indexes, fp_out=None, q_bits=8, q_mantisa_bits=3, scale=None):
        """Dequantize only rows ``indexes`` of a [rows, cols] quantized matrix (cols multiple of group_size)."""
        s = scale if scale is not None else self.scale
        rows = self.orig_shape[0] if self.orig_shape is not None else input_q.shape[0]
        qr = input_q.reshape(rows, -1)[indexes]
        sr = s.reshape(rows, -1)[indexes]
        y = self._deq(qr.reshape(-1), sr.reshape(-1), q_bits, q_mantisa_bits).view(len(indexes), -1)
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


# ----------------------------------------------------------------------------------------
# FP6 / FP12 (and generic E/M) minifloat group quantization with bit packing (csrc/kernels/fpq.hip)
# ----------------------------------------------------------------------------------------
def _mini_fmt(q_bits, mantissa_bits):
    ebits = q_bits - 1 - mantissa_bits
    assert q_bits in (6, 8, 12) and ebits >= 2 and mantissa_bits >= 1, f"unsupported FP{q_bits} e{ebits}m{mantissa_bits}"
    bias = 2**(ebits - 1) - 1
    maxval = (2.0 - 2.0**-mantissa_bits) * 2.0**((2**ebits - 1) - bias)
    return ebits, bias, maxval


def _ref_encode(x, q_bits, mbits, stochastic=False, gen=None):
    """fp32 values (already scaled into range) -> integer codes sign|exp|mant (saturating, no inf/nan)."""
    ebits, bias, maxval = _mini_fmt(q_bits, mbits)
    sign = (x < 0).to(torch.int32)
    a = x.abs().clamp(max=maxval)
    _, k = torch.frexp(a)
    e = k.to(torch.int32) - 1
    emin = 1 - bias
    msc = 2.0**mbits
    u = torch.rand(a.shape, generator=gen) if stochastic else None
    rnd = (lambda t: torch.floor(t + u)) if stochastic else torch.round  # torch.round = half-to-even
    sub = e < emin
    mf_sub = torch.ldexp(a, torch.tensor(mbits - emin, dtype=torch.int32))
    mf_nrm = (torch.ldexp(a, -e) - 1.0) * msc
    m = torch.where(sub, rnd(mf_sub), rnd(mf_nrm))
    ef = torch.where(sub, torch.zeros_like(e), e + bias)
    carry = m >= msc
    ef = torch.where(carry, ef + 1, ef)
    m = torch.where(carry, torch.zeros_like(m), m)
    sat = ef > (2**ebits - 1)
    ef = torch.where(sat, torch.full_like(ef, 2**ebits - 1), ef)
    m = torch.where(sat, torch.full_like(m, msc - 1), m)
    code = (sign << (ebits + mbits)) | (ef << mbits) | m.to(torch.int32)
    return torch.where(a > 0, code, sign << (ebits + mbits))


def _ref_decode(code, q_bits, mbits):
    ebits, bias, _ = _mini_fmt(q_bits, mbits)
    code = code.to(torch.int32)
    mant = (code & (2**mbits - 1)).float()
    ef = (code >> mbits) & (2**ebits - 1)
    neg = ((code >> (ebits + mbits)) & 1).bool()
    sub = torch.ldexp(mant, torch.tensor(1 - bias - mbits, dtype=torch.int32))
    nrm = torch.ldexp(1.0 + mant / 2**mbits, ef - bias)
    v = torch.where(ef == 0, sub, nrm)
    return torch.where(neg, -v, v)


def _pack(codes, bits):
    c = codes.reshape(-1, 4).to(torch.int64)
    if bits == 8:
        return c.to(torch.uint8).reshape(-1)
    if bits == 6:
        w = c[:, 0] | (c[:, 1] << 6) | (c[:, 2] << 12) | (c[:, 3] << 18)
        return torch.stack([w & 255, (w >> 8) & 255, (w >> 16) & 255], 1).to(torch.uint8).reshape(-1)
    w0, w1 = c[:, 0] | (c[:, 1] << 12), c[:, 2] | (c[:, 3] << 12)
    return torch.stack([w0 & 255, (w0 >> 8) & 255, (w0 >> 16) & 255, w1 & 255, (w1 >> 8) & 255, (w1 >> 16) & 255],
                       1).to(torch.uint8).reshape(-1)


def _unpack(q, bits):
    b = q.to(torch.int64)
    if bits == 8:
        return b
    if bits == 6:
        b = b.reshape(-1, 3)
        w = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        return torch.stack([w & 63, (w >> 6) & 63, (w >> 12) & 63, (w >> 18) & 63], 1).reshape(-1)
    b = b.reshape(-1, 6)
    w0, w1 = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16), b[:, 3] | (b[:, 4] << 8) | (b[:, 5] << 16)
    return torch.stack([w0 & 4095, w0 >> 12, w1 & 4095, w1 >> 12], 1).reshape(-1)


def quantize_minifloat(x, group_size=512, q_bits=6, mantissa_bits=2, stochastic=False, seed=0):
    """Returns (packed uint8 [numel * q_bits / 8], scales fp32 [groups]). FP6 e3m2 by default."""
    x = x.contiguous()
    ng = _groups(x, group_size)
    ebits, _, maxval = _mini_fmt(q_bits, mantissa_bits)
    assert group_size % 4 == 0
    if native.use_native(x):
        q = torch.empty(x.numel() * q_bits // 8, dtype=torch.uint8, device=x.device)
        scales = torch.empty(ng, dtype=torch.float32, device=x.device)
        native.check(native.kernels().hds_quant_minifloat(native.dt(x), x.data_ptr(), q.data_ptr(), scales.data_ptr(),
                                                          ng, group_size, ebits, mantissa_bits, int(stochastic),
                                                          int(seed) & 0x7FFFFFFF, native.stream()), "quant_minifloat")
        return q, scales
    g = x.float().reshape(-1, group_size)
    amax = g.abs().amax(1)
    scale = torch.where(amax > 0, amax / maxval, torch.ones_like(amax))
    gen = torch.Generator().manual_seed(int(seed)) if stochastic else None
    codes = _ref_encode(g / scale[:, None], q_bits, mantissa_bits, stochastic, gen)
    return _pack(codes, q_bits), scale


def dequantize_minifloat(q, scales, group_size=512, q_bits=6, mantissa_bits=2, dtype=torch.bfloat16, out=None):
    ng = scales.numel()
    ebits, _, _ = _mini_fmt(q_bits, mantissa_bits)
    if native.use_native(q):
        y = out if out is not None else torch.empty(ng * group_size, dtype=dtype, device=q.device)
        native.check(native.kernels().hds_dequant_minifloat(native.dt(y), q.data_ptr(), scales.data_ptr(),
                                                            y.data_ptr(), ng, group_size, ebits, mantissa_bits,
                                                            native.stream()), "dequant_minifloat")
        return y
    v = _ref_decode(_unpack(q, q_bits), q_bits, mantissa_bits).reshape(-1, group_size) * scales[:, None].float()
    y = v.reshape(-1).to(dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def fp6_linear(x, q_weight, scales, out_features, in_features, group_size, mantissa_bits=2):
    """y = x @ dequant(W)^T for an FP6-packed weight [out, in] (row-major, groups along ``in``).

    Decode-sized inputs (<= 8 rows) run the fused HIP GEMV that reads 6-bit weights straight from HBM; larger
    batches dequantize the weight once to bf16 and use the matrix cores (hipBLASLt)."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, in_features)
    M = x2.shape[0]
    if not _needs_grad(x2) and native.use_native(x2) and M <= 8 and x2.dtype == torch.bfloat16 \
            and in_features % 16 == 0 \
            and group_size % 16 == 0:
        x2 = x2.contiguous()
        y = torch.empty(M, out_features, dtype=torch.bfloat16, device=x.device)
        native.check(native.kernels().hds_fp6_gemv(x2.data_ptr(), q_weight.data_ptr(), scales.data_ptr(),
                                                   y.data_ptr(), M, out_features, in_features, group_size,
                                                   5 - mantissa_bits, mantissa_bits, native.stream()), "fp6_gemv")
        return y.view(*lead, out_features)
    if wmix_eligible(x2, out_features, in_features, group_size):  # batched decode / chunked prefill: MFMA
        return wmix_gemm(x2, q_weight, scales, out_features, in_features, group_size, "fp6",
                         5 - mantissa_bits).view(*lead, out_features)
    w = dequantize_minifloat(q_weight, scales, group_size, 6, mantissa_bits, x.dtype).view(out_features, in_features)
    return torch.nn.functional.linear(x, w)
