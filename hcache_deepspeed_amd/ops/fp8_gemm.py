"""MX-FP8 GEMM: OCP e4m3 elements with one e8m0 (power-of-two) scale per 32 elements along K, multiplied on the
block-scaled matrix-core op of CDNA4 (csrc/kernels/gemm.hip ``gemm_mxfp8_kernel``, 2x the bf16 MFMA rate).

Reference parity: deepspeed/ops/fp_quantizer/fp8_gemm.py ``matmul_fp8`` (bf16 activations x group-quantized
FP8 weights, dequantized inside a Triton GEMM). On MI355X the hardware multiplies scaled FP8 directly, so both
operands are quantized to MX-FP8 (activations on the fly, per 32-element block -- finer than the reference's
weight groups) and nothing is dequantized in the inner loop.

Layout of an MX tensor ``(q, s)`` for a logical [R, K] matrix (K % 128 == 0):
  * ``q``: uint8 [R, K] -- e4m3 bit patterns;
  * ``s``: uint8 [K/128, R, 4] -- e8m0 scale of block (r, 4*t + g) at ``s[t, r, g]`` (tile-major, so one K-tile
    of 256 rows is one contiguous KiB for the kernel's LDS-DMA).
Value = e4m3(q) * 2**(s - 127).
"""
import torch

from . import native

E4M3_MAX = 448.0
E4M3_EMAX = 8


def _native(x):
    return native.use_native(x)


def mx_quantize_ref(x):
    """Torch reference of the quantizer (CPU path and numerics reference)."""
    R, K = x.shape
    assert K % 128 == 0, "MX-FP8: K must be a multiple of 128"
    xb = x.float().reshape(R, K // 32, 32)
    amax = xb.abs().amax(-1)
    ex = torch.where(amax > 0, torch.floor(torch.log2(amax.clamp_min(1e-38))) - E4M3_EMAX,
                     torch.full_like(amax, -127.0)).clamp(-127, 127)
    scaled = (xb * torch.exp2(-ex).unsqueeze(-1)).clamp(-E4M3_MAX, E4M3_MAX)
    q = scaled.to(torch.float8_e4m3fn).view(torch.uint8).reshape(R, K)
    s = (ex + 127).to(torch.uint8).reshape(R, K // 128, 4).permute(1, 0, 2).contiguous()
    return q, s


def mx_quantize(x):
    """bf16 [R, K] -> (q uint8 [R, K], s uint8 [K/128, R, 4])."""
    assert x.dim() == 2 and x.shape[1] % 128 == 0
    if not (_native(x) and x.dtype == torch.bfloat16 and x.stride(1) == 1 and x.stride(0) % 8 == 0):
        return mx_quantize_ref(x)
    R, K = x.shape
    q = torch.empty(R, K, dtype=torch.uint8, device=x.device)
    s = torch.empty(K // 128, R, 4, dtype=torch.uint8, device=x.device)
    native.check(native.kernels().hds_mx_quant(x.data_ptr(), q.data_ptr(), s.data_ptr(), R, K, x.stride(0),
                                               native.stream()), "mx_quant")
    return q, s


def mx_dequantize(q, s, dtype=torch.float32):
    R, K = q.shape
    v = q.view(torch.float8_e4m3fn).float().reshape(R, K // 32, 32)
    sc = torch.exp2(s.permute(1, 0, 2).reshape(R, K // 32).float() - 127.0)
    return (v * sc.unsqueeze(-1)).reshape(R, K).to(dtype)


VARIANT = int(__import__("os").environ.get("HDS_GEMM_VARIANT", "1"))


def mx_gemm(qa, sa, qb, sb, alpha=1.0, out=None, variant=None):
    """bf16 [M, N] = alpha * dequant(qa, sa) @ dequant(qb, sb).T."""
    M, K = qa.shape
    N = qb.shape[0]
    ok = (_native(qa) and native.kernels().hds_gemm_mxfp8_supported(M, N, K, qa.stride(0), qb.stride(0), N)
          and qa.is_contiguous() and qb.is_contiguous() and sa.is_contiguous() and sb.is_contiguous())
    if not ok:
        r = (mx_dequantize(qa, sa) @ mx_dequantize(qb, sb).t()) * alpha
        r = r.to(torch.bfloat16)
        return r if out is None else out.copy_(r)
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=qa.device)
    native.check(native.kernels().hds_gemm_mxfp8(qa.data_ptr(), sa.data_ptr(), qb.data_ptr(), sb.data_ptr(),
                                                 out.data_ptr(), M, N, K, qa.stride(0), qb.stride(0), out.stride(0),
                                                 float(alpha), VARIANT if variant is None else int(variant),
                                                 native.stream()), "gemm_mxfp8")
    return out


def mx_supported(M, N, K):
    return M % 256 == 0 and N % 256 == 0 and K % 256 == 0


def fp8_linear(x, wq, ws, bias=None):
    """F.linear with an MX-FP8 weight (wq [N, K], ws): activations are MX-quantized on the fly."""
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    M, K = x2.shape
    N = wq.shape[0]
    if not mx_supported(M, N, K):
        r = x2.float() @ mx_dequantize(wq, ws).t()
        r = r.to(x.dtype)
    else:
        qa, sa = mx_quantize(x2.to(torch.bfloat16).contiguous())
        r = mx_gemm(qa, sa, wq, ws).to(x.dtype)
    if bias is not None:
        r = r + bias
    return r.reshape(*shp[:-1], N)
