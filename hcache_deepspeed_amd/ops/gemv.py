"""Decode-sized bf16 linear on the HIP GEMV (csrc/kernels/gemv.hip): ``linear(x, w, b)`` equals ``F.linear`` and
takes the GEMV path when x has at most 8 rows and the shape is one where the weight stream is faster than
hipBLASLt's small-M GEMM (``profiles/gemv_bench_r2.jsonl``); everything else goes to ``F.linear``."""
import torch
import torch.nn.functional as F

from . import native

# Weight sizes (elements) that take the GEMV. At M = 1 every size does: in a real decode step (weights streamed from
# HBM, not re-read from the 256 MB MALL as in a micro-benchmark loop) the GEMV beats hipBLASLt's small-M GEMM on the
# gate_up projection and the LM head as well -- Llama-3-8B v2 decode 234.8 vs 211.0 tok/s at B = 1, same box
# (profiles/r3/v2_decode_gemv_rule_r3.jsonl). Its dot products make it VALU-bound as M grows (M = 4: qkv 1.4x,
# down 0.73x; M = 8: o 1.36x, qkv 0.98x, gate_up a loss in decode: 1124 vs 1462 tok/s at B = 8), so beyond one row
# the limit is 32M elements up to M = 4 and 16M up to M = 8 (profiles/gemv_bench_r2.jsonl).
_os = __import__("os")
MAX_GEMV_NUMEL_M1 = int(_os.environ.get("HDS_GEMV_MAX_NUMEL_M1", str(1 << 40)))
MAX_GEMV_NUMEL = int(_os.environ.get("HDS_GEMV_MAX_NUMEL", str(64 * 1024 * 1024)))


def max_numel(M):
    return MAX_GEMV_NUMEL_M1 if M == 1 else MAX_GEMV_NUMEL >> (1 if M <= 4 else 2)


def gemv_ok(x2, w, b=None):
    if not (native.use_native(x2) and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2):
        return False
    M, K = x2.shape
    N = w.shape[0]
    if M > 8 or w.shape[1] != K or not w.is_contiguous() or x2.stride(1) != 1 or x2.stride(0) % 8:
        return False
    if x2.data_ptr() % 16 or w.data_ptr() % 16 or N * K > max_numel(M):
        return False
    if b is not None and (b.dtype != torch.bfloat16 or not b.is_contiguous()):
        return False
    return bool(native.kernels().hds_gemv_bf16_supported(M, N, K))


def gemv(x2, w, b=None):
    M, K = x2.shape
    N = w.shape[0]
    y = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
    native.check(native.kernels().hds_gemv_bf16(x2.data_ptr(), w.data_ptr(), native.ptr(b), y.data_ptr(), M, N, K,
                                                x2.stride(0), N, native.stream()), "gemv_bf16")
    return y


# 2..16 token rows: the matrix-core skinny GEMM (csrc/kernels/gemv.hip skinny_mfma_kernel) instead of the VALU GEMV /
# hipBLASLt's small-M tiles (HDS_SKINNY_GEMM=0: those)
SKINNY = _os.environ.get("HDS_SKINNY_GEMM", "1") == "1"
SKINNY_MIN_M = int(_os.environ.get("HDS_SKINNY_MIN_M", "2"))  # 1: one-row linears too (instead of the VALU GEMV)


def skinny_ok(x2, w, b=None):
    if not (SKINNY and native.use_native(x2) and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and w.dim() == 2):
        return False
    M, K = x2.shape
    if not SKINNY_MIN_M <= M <= 16 or w.shape[1] != K or K % 128 or not w.is_contiguous() or x2.stride(1) != 1 or x2.stride(0) % 8:
        return False
    if x2.data_ptr() % 16 or w.data_ptr() % 16:
        return False
    return b is None or (b.dtype == torch.bfloat16 and b.is_contiguous())


def skinny(x2, w, b=None):
    M, K = x2.shape
    N = w.shape[0]
    y = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
    native.check(native.kernels().hds_skinny_gemm_bf16(x2.data_ptr(), w.data_ptr(), native.ptr(b), y.data_ptr(), M, N,
                                                       K, x2.stride(0), N, native.stream()), "skinny_gemm_bf16")
    return y


def linear(x, w, b=None):
    """``F.linear(x, w, b)``; decode-sized bf16 inputs run the HIP GEMV (one row) or the skinny matrix-core GEMM
    (2..16 rows)."""
    if x.dim() >= 1 and x.is_cuda:
        x2 = x.reshape(-1, x.shape[-1])
        if skinny_ok(x2, w, b):
            return skinny(x2, w, b).view(*x.shape[:-1], w.shape[0])
        if gemv_ok(x2, w, b):
            return gemv(x2, w, b).view(*x.shape[:-1], w.shape[0])
    return F.linear(x, w, b)


def fused_ok(h2, w, gamma=None, glu=False):
    """Can ``fused_gemv`` take these decode rows on the HIP kernel (bf16, <= 8 rows, 16-B aligned rows)?"""
    if not (native.use_native(h2) and h2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2):
        return False
    M, K = h2.shape
    if M > 8 or w.shape[1] != K or K % 8 or not w.is_contiguous() or h2.stride(1) != 1 or h2.stride(0) != K:
        return False
    if glu and w.shape[0] % 2:
        return False
    if gamma is not None and (gamma.dtype != torch.bfloat16 or not gamma.is_contiguous() or gamma.numel() != K):
        return False
    return h2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and w.numel() <= max_numel(M)


def _unfused(h2, w, res, gamma, eps, glu):
    from .activations import glu as _glu
    from .norm import rms_norm
    r, x = h2, h2
    if gamma is not None:
        if res is None:
            x = rms_norm(h2, gamma, eps)
        else:
            x, r = rms_norm(h2, gamma, eps, res)
    y = linear(x, w)
    return (_glu(y, "silu") if glu else y), r, x


def fused_gemv(h, w, res=None, gamma=None, eps=1e-5, glu=False, want_x=False, x_out=None):
    """Decode projection with the pre-norm and / or the gated activation folded in (csrc/kernels/gemv.hip
    ``hds_gemv_fused_bf16``). With ``gamma``: the rows are RMSNorm(h + res) * gamma -- the new residual ``h + res`` is
    returned too (``h`` itself without ``res``), and the normed rows when ``want_x`` (HCache hidden latents). With
    ``glu``: ``w`` is [gate; up] and the result is silu(x . gate^T) * (x . up^T). Returns (y, residual, x or None);
    rows or weights the fused kernel does not take run the unfused kernels (the same arithmetic). ``x_out``: a
    contiguous [rows, K] buffer the normed rows are written into (``want_x``; the unfused fallback returns its own)."""
    shape = h.shape
    h2 = h.reshape(-1, shape[-1])
    res2 = None if res is None else res.reshape(-1, shape[-1])
    N = w.shape[0] // 2 if glu else w.shape[0]
    ok = (fused_ok(h2, w, gamma, glu) and (gamma is not None or glu)
          and (res2 is None or (res2.dtype == h2.dtype and res2.stride() == h2.stride() and res2.data_ptr() % 16 == 0)))
    if not ok:  # the unfused kernels (GEMV or hipBLASLt by the size rules, RMSNorm, GLU): the model's other path
        y, r, x = _unfused(h2, w, res2, gamma, eps, glu)
    else:
        M, K = h2.shape
        y = torch.empty(M, N, dtype=h2.dtype, device=h2.device)
        r = h2 if res2 is None else torch.empty_like(h2)  # never in place: other workgroups still read res
        x = None
        if want_x and gamma is not None:
            ok_out = (x_out is not None and x_out.dtype == h2.dtype and x_out.is_contiguous()
                      and x_out.numel() == h2.numel() and x_out.data_ptr() % 16 == 0)
            x = x_out.view(h2.shape) if ok_out else torch.empty_like(h2)
        native.check(native.kernels().hds_gemv_fused_bf16(
            h2.data_ptr(), native.ptr(res2), native.ptr(gamma), float(eps), w.data_ptr(), y.data_ptr(),
            native.ptr(r if res2 is not None else None), native.ptr(x), int(bool(glu)), M, N, K, K, N,
            native.stream()), "gemv_fused_bf16")
        if gamma is None:
            x = h2
    lead = shape[:-1]
    return (y.view(*lead, N), r.view(shape), None if x is None or not want_x else x.view(shape))
