"""Hand-written MFMA GEMM for the transformer projection shapes (csrc/kernels/gemm.hip).

``gemm_nt(a, b)`` computes ``a @ b.T`` -- exactly ``F.linear(a, b)`` for a weight ``b`` of shape [out, in] --
with bf16 operands and fp32 accumulation, optionally scaled and accumulated into ``out``. Shapes outside
the kernel's tiling (M, N multiples of 256, K a multiple of 128) go to ``torch.matmul`` (hipBLASLt).
"""
import os

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


# ----------------------------------------------------------------------------------------------------------------
# weight-gradient GEMM layout: dW[N, K] (+)= dY[T, N]^T X[T, K]
# ----------------------------------------------------------------------------------------------------------------
# 1: 64x64 tile, 2-B LDS ops; 2: 64x128, 8/16-B LDS ops -- the same ~4.5-5 TB/s at the step's shapes
# (profiles/r3/transpose_bench_r3.log): HBM read/write mix, not LDS, bounds both
_TRANSPOSE_VAR = int(os.environ.get("HDS_TRANSPOSE_VAR", "1"))


def transpose2d(x, variant=None):
    """[R, C] (unit last stride) -> contiguous [C, R]; HIP LDS-tiled kernel for bf16 on the GPU."""
    R, C = x.shape
    if not (native.use_native(x) and x.dtype == torch.bfloat16 and x.stride(1) == 1 and R % 8 == 0
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0):
        return x.t().contiguous()
    out = torch.empty(C, R, dtype=x.dtype, device=x.device)
    var = _TRANSPOSE_VAR if variant is None else int(variant)
    native.check(native.kernels().hds_transpose_bf16_var(x.data_ptr(), out.data_ptr(), R, C, x.stride(0), var,
                                                         native.stream()), "transpose_bf16")
    return out


_WGRAD_LAYOUT = os.environ.get("HDS_WGRAD_LAYOUT", "auto")  # auto | direct | nt | direct_sk2 | nt_sk2
_WGRAD_CHOICE = {}
_SPLITK = os.environ.get("HDS_WGRAD_SPLITK", "0") == "1"  # two-stream split-K candidates in the timed choice
_B2 = os.environ.get("HDS_WGRAD_B2", "1") == "1"  # batched two-half split-K candidates in the timed choice


def _mm_into(out, a, bt, accumulate):
    if out.dtype == a.dtype:
        if accumulate:
            out.addmm_(a, bt)
        else:
            torch.mm(a, bt, out=out)
    else:  # fp32 accumulator from bf16 operands
        if accumulate:
            torch.addmm(out, a, bt, out_dtype=out.dtype, out=out)
        else:
            torch.mm(a, bt, out_dtype=out.dtype, out=out)


_SIDE = {}


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(dev)
    return s


def _bmm_halves(out, a, bt, accumulate):
    """out (+)= a[N, T] @ bt[T, K] as ONE batched GEMM over the two halves of the token (reduction) dimension into
    fp32 partials [2, N, K], then one add. Batch 2 doubles the output-tile count of the grid (qkv: 384 -> 768 tiles of
    256^2 = 3 full waves on 256 CUs instead of 1.5; down: 896 -> 1792 = 7 instead of 3.5) without a second stream."""
    N, T = a.shape
    K = bt.shape[1]
    h = T // 2
    A = a.as_strided((2, N, h), (h * a.stride(1), a.stride(0), a.stride(1)), a.storage_offset())
    B = bt.as_strided((2, h, K), (h * bt.stride(0), bt.stride(0), bt.stride(1)), bt.storage_offset())
    part = torch.bmm(A, B, out_dtype=torch.float32) if out.is_cuda else torch.bmm(A.float(), B.float())
    if accumulate:
        out.add_(part[0] + part[1])
    else:
        torch.add(part[0], part[1], out=out)


def _wgrad_run(layout, dy2, x2, out, accumulate, dyt=None, xt=None):
    """``layout``: "direct" (TN as autograd issues it), "nt" (HIP transposes + the NT GEMM), or either with "_sk2":
    the token (reduction) dimension split in two halves run as CONCURRENT GEMMs on two streams, the second into a
    scratch buffer added at the join, or with "_b2": the two halves as one batched GEMM (``_bmm_halves``). A
    projection with few output tiles (qkv: 24 x 16 tiles of 256 = 1.5 waves on 256 CUs; down: 3.5 waves) otherwise
    idles part of the chip in its last wave; two half-K GEMMs in flight fill it. ``dyt`` / ``xt``: transposes the
    producer already wrote ([N, T] / [K, T]); the "nt" forms use them instead of transposing (``x2`` may then be
    None)."""
    base, sk2, b2 = layout.split("_")[0], layout.endswith("_sk2"), layout.endswith("_b2")
    if base == "nt":  # hipBLASLt's NT form on transposed copies (the forward GEMM's fast layout)
        a = dyt if dyt is not None else transpose2d(dy2)
        bt = (xt if xt is not None else transpose2d(x2)).t()
    else:
        a, bt = dy2.t(), x2
    split_a, split_b = (lambda t, lo, hi: t[:, lo:hi]), (lambda t, lo, hi: t[lo:hi])
    if b2 and a.shape[1] % 2 == 0:
        _bmm_halves(out, a, bt, accumulate)
        return
    if not sk2 or not out.is_cuda:
        _mm_into(out, a, bt, accumulate)
        return
    T = a.shape[1]
    h = (T // 2) // 256 * 256 or T // 2
    cur = torch.cuda.current_stream(out.device)
    side = _side_stream(out.device)
    tmp = torch.empty_like(out)
    side.wait_stream(cur)
    _mm_into(out, split_a(a, 0, h), split_b(bt, 0, h), accumulate)
    with torch.cuda.stream(side):
        _mm_into(tmp, split_a(a, h, T), split_b(bt, h, T), False)
        for t in (a, bt, tmp):
            t.record_stream(side)
    cur.wait_stream(side)
    out.add_(tmp)


def _time_layout(layout, dy2, x2, out, accumulate, dyt=None, xt=None, reps=2):
    """Milliseconds of one layout; inf when its scratch (output copy, transposes) does not fit: a near-full device
    (large micro-batches, offloaded optimizer states) must not fail in the autotuner."""
    try:
        scratch = torch.zeros_like(out)
        _wgrad_run(layout, dy2, x2, scratch, accumulate, dyt, xt)  # warm (hipBLASLt solution lookup, allocator)
    except torch.OutOfMemoryError:
        return float("inf")
    best = float("inf")
    for _ in range(reps):  # min of reps: one timed run mis-picked the down-projection layout in situ
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _wgrad_run(layout, dy2, x2, scratch, accumulate, dyt, xt)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def _b2_useful(N, K):
    """A two-half batched GEMM only pays when the 256 x 256 output-tile grid leaves the last wave of 256 CUs about
    half empty (qkv 1.5 waves, down 3.5; not gate_up 7 or o 1)."""
    tiles = -(-N // 256) * -(-K // 256)
    frac = (tiles % 256) / 256
    return _B2 and 0.2 < frac < 0.8


def _rows_bucket(t):
    """Token-row count as the layout tuners key it: rounded up to 2048, so GEMMs whose row count moves a little
    from step to step (MoE experts over their occupied capacity slots) reuse one timing instead of re-timing every
    new size inside the step."""
    return -(-int(t) // 2048) * 2048


_NT_BY_N = {}  # dy columns -> True if the timed choice for that gradient width was an "nt" form


def wants_transposed_dy(n):
    """Should a producer of a [T, n] output gradient also write its transpose (ops/activations.glu)? Yes until a
    weight gradient of that width has chosen a non-NT layout."""
    return _NT_BY_N.get(int(n), True)


def wgrad(dy2, x2, out, accumulate=False, dyt=None, xt=None):
    """out[N, K] (+)= dy2[T, N]^T @ x2[T, K] with the fastest layout for this shape: the TN GEMM autograd issues
    (``direct``), two HBM-rate HIP transposes + the NT GEMM (``nt``), or either as one batched GEMM over the two
    token halves (``_b2``, shapes whose tile grid ends in a half-empty wave). ``HDS_WGRAD_LAYOUT=auto`` times the
    candidates once per (shape, dtype, accumulate, pre-transposed operands) on the first call
    (profiles/wgrad_layout_r2.log: NT runs 1.44-1.47 PF/s where TN runs 0.94-1.10 at the o / gate_up shapes).
    ``dyt`` [N, T] / ``xt`` [K, T]: transposes the producers already wrote (glu, runtime/zero/linear.py); with
    ``x2`` None only the NT forms are possible."""
    layout = _WGRAD_LAYOUT
    T, N = dy2.shape
    K = xt.shape[0] if x2 is None else x2.shape[1]
    if layout == "auto":
        if not (dy2.is_cuda and dy2.dtype == torch.bfloat16 and (x2 is None or x2.dtype == torch.bfloat16)
                and dy2.stride(1) == 1 and (x2 is None or x2.stride(1) == 1)):
            layout = "direct" if x2 is not None else "nt"
        else:
            key = (_rows_bucket(T), N, K, out.dtype, bool(accumulate), x2 is None, dyt is not None)
            layout = _WGRAD_CHOICE.get(key)
            if layout is None:
                b2 = ("_b2", ) if _b2_useful(N, K) else ()
                if x2 is None:
                    cands = ("nt", ) + tuple("nt" + x for x in b2)
                else:
                    cands = ("direct", "nt") + tuple(c + x for x in b2 for c in ("direct", "nt")) + (
                        ("direct_sk2", "nt_sk2") if _SPLITK else ())
                times = {c: _time_layout(c, dy2, x2, out, accumulate, dyt, xt) for c in cands}
                layout = min(times, key=times.get)
                if x2 is not None and layout != "direct" and times[layout] > 0.97 * times["direct"]:
                    layout = "direct"  # within noise: keep the plain form
                if times[layout] == float("inf"):  # nothing fit: the plain form now, time again on a later call
                    layout = "direct" if x2 is not None else "nt"
                else:
                    _WGRAD_CHOICE[key] = layout
                    _NT_BY_N[N] = layout.startswith("nt")
    elif x2 is None and not layout.startswith("nt"):
        layout = "nt"
    _wgrad_run(layout, dy2, x2, out, accumulate, dyt, xt)
    return out


# ----------------------------------------------------------------------------------------------------------------
# input-gradient GEMM layout: dX[T, K] = dY[T, N] W[N, K]
# ----------------------------------------------------------------------------------------------------------------
_DGRAD_LAYOUT = os.environ.get("HDS_DGRAD_LAYOUT", "auto")  # auto | direct | nt
_DGRAD_CHOICE = {}


def _dgrad_run(layout, dy2, w, out, cache=None):
    if layout == "nt":  # nt: dY @ (W^T)^T, hipBLASLt's NT form
        b = cache.get("wt") if cache is not None else None
        if b is None:
            b = transpose2d(w).t()
            if cache is not None:
                cache["wt"] = b
    else:
        b = w
    if out is None:
        return torch.mm(dy2, b)
    return torch.mm(dy2, b, out=out)


def dgrad(dy2, w, out=None, cache=None):
    """dy2[T, N] @ w[N, K] with the faster of the NN GEMM autograd issues and a HIP transpose of the (small) weight +
    the NT GEMM, timed once per shape under ``HDS_DGRAD_LAYOUT=auto`` (the NT form ran 1.51-1.59 PF/s against
    1.32-1.39 for NN at the bench shapes, profiles/gemm_layouts_r1.log). ``cache``: a dict the caller keeps for the
    calls that share ``w`` (the fused CE's per-chunk LM-head dgrads): the transposed weight is made once."""
    layout = _DGRAD_LAYOUT
    if layout == "auto":
        if not (dy2.is_cuda and dy2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and dy2.stride(1) == 1
                and w.stride(1) == 1):
            layout = "direct"
        else:
            key = (_rows_bucket(dy2.shape[0]), dy2.shape[1], tuple(w.shape))
            layout = _DGRAD_CHOICE.get(key)
            if layout is None:
                times = {}
                for cand in ("direct", "nt"):
                    try:  # a near-full device: a candidate whose scratch does not fit is out
                        _dgrad_run(cand, dy2, w, None)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        _dgrad_run(cand, dy2, w, None)
                        e1.record()
                        e1.synchronize()
                        times[cand] = e0.elapsed_time(e1)
                    except torch.OutOfMemoryError:
                        times[cand] = float("inf")
                layout = "nt" if times["nt"] < 0.97 * times["direct"] else "direct"
                if min(times.values()) < float("inf"):
                    _DGRAD_CHOICE[key] = layout
    return _dgrad_run(layout, dy2, w, out, cache)
