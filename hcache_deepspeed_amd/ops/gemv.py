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


def linear(x, w, b=None):
    """``F.linear(x, w, b)``; decode-sized bf16 inputs run the HIP GEMV."""
    if x.dim() >= 1 and x.is_cuda:
        x2 = x.reshape(-1, x.shape[-1])
        if gemv_ok(x2, w, b):
            return gemv(x2, w, b).view(*x.shape[:-1], w.shape[0])
    return F.linear(x, w, b)
