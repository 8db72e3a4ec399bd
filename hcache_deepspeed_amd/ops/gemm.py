"""Hand-written MFMA GEMM for the transformer projection shapes (csrc/kernels/gemm.hip).

``gemm_nt(a, b)`` computes ``a @ b.T`` -- exactly ``F.linear(a, b)`` for a weight ``b`` of shape [out, in] --
with bf16 operands and fp32 accumulation, optionally scaled and accumulated into ``out``. Shapes outside
the kernel's tiling (M, N multiples of 256, K a multiple of 128) go to ``torch.matmul`` (hipBLASLt).
"""
import torch

from . import native


def _native_ok(a, b, out):
    if not (native.use_native(a) and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2
            and b.dim() == 2 and a.stride(1) == 1 and b.stride(1) == 1 and a.shape[1] == b.shape[1]):
        return False
    if out is not None and (out.dtype != torch.bfloat16 or out.stride(1) != 1 or
                            tuple(out.shape) != (a.shape[0], b.shape[0])):
        return False
    M, K = a.shape
    N = b.shape[0]
    ldc = N if out is None else out.stride(0)
    return bool(native.kernels().hds_gemm_nt_supported(M, N, K, a.stride(0), b.stride(0), ldc))


def gemm_nt_supported(M, N, K):
    return M % 256 == 0 and N % 256 == 0 and K % 128 == 0 and M > 0 and N > 0 and K > 0


VARIANT = int(__import__("os").environ.get("HDS_GEMM_VARIANT", "1"))  # 0 plain, 1 staggered wave groups


def gemm_nt(a, b, out=None, alpha=1.0, accumulate=False, variant=None):
    """out (+)= alpha * a @ b.T for 2-D a [M, K], b [N, K]."""
    if not _native_ok(a, b, out):
        r = torch.matmul(a, b.t())
        if alpha != 1.0:
            r = r * alpha
        if out is None:
            return r
        if accumulate:
            out.add_(r.to(out.dtype))
        else:
            out.copy_(r)
        return out
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=a.dtype, device=a.device)
    native.check(native.kernels().hds_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0),
                                              b.stride(0), out.stride(0), float(alpha), int(bool(accumulate)),
                                              VARIANT if variant is None else int(variant), native.stream()),
                 "gemm_nt")
    return out
