"""Decode-sized bf16 linear on the HIP GEMV (csrc/kernels/gemv.hip): ``linear(x, w, b)`` equals ``F.linear`` and
takes the GEMV path when x has at most 8 rows and the shape is one where the weight stream is faster than
hipBLASLt's small-M GEMM (``profiles/gemv_bench_r2.jsonl``); everything else goes to ``F.linear``."""
import torch
import torch.nn.functional as F

from . import native

# weights up to this many elements take the GEMV (hipBLASLt is latency-bound below it at M <= 8)
MAX_GEMV_NUMEL = int(__import__("os").environ.get("HDS_GEMV_MAX_NUMEL", "0"))  # set from the GPU measurement


def gemv_ok(x2, w, b=None):
    if not (native.use_native(x2) and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2):
        return False
    M, K = x2.shape
    N = w.shape[0]
    if M > 8 or w.shape[1] != K or not w.is_contiguous() or x2.stride(1) != 1 or x2.stride(0) % 8:
        return False
    if x2.data_ptr() % 16 or w.data_ptr() % 16 or N * K > MAX_GEMV_NUMEL:
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


def linear(x, w, b=None):
    """``F.linear(x, w, b)``; decode-sized bf16 inputs run the HIP GEMV."""
    if x.dim() >= 1 and x.is_cuda:
        x2 = x.reshape(-1, x.shape[-1])
        if gemv_ok(x2, w, b):
            return gemv(x2, w, b).view(*x.shape[:-1], w.shape[0])
    return F.linear(x, w, b)
