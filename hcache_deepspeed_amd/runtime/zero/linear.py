"""ZeRO linear Functions (reference runtime/zero/linear.py ``LinearFunctionForZeroStage3`` :50).

Two jobs:

* memory efficiency (ZeRO-3): save the input and the Parameter OBJECT, not the weight tensor (below);
* in-place weight gradients (every stage, ``mi355x.direct_wgrad``): the weight gradient GEMM writes straight
  into the parameter's slice of the flat ZeRO gradient buffer -- ``mm(out=grad)`` on the first micro-step of
  a window, ``addmm_(beta=1)`` after -- so neither the per-step zero fill of the gradient buffer nor autograd's
  AccumulateGrad add (``grad += dW``: a full read-modify-write of every weight gradient) runs. Readiness
  bookkeeping stays with the parameter's post-accumulate hook, which autograd still fires (with no gradient).


A plain ``F.linear`` saves the weight TENSOR for backward, which pins the gathered full buffer of the whole
unit until the backward pass -- a partitioned model would keep every layer's gathered weights alive. This
Function saves only the input and keeps a reference to the Parameter OBJECT; by the time its backward runs
the unit has been re-gathered (pre-backward hook) and ``weight.data`` points at the new full buffer, so the
forward copy can be freed right after the layer's forward.
"""
import types

import torch
import torch.nn as nn
import torch.nn.functional as F


def write_weight_grad(w, compute):
    """If ZeRO owns ``w``'s gradient buffer and allows in-place writes, call ``compute(out, accumulate)`` to
    produce the weight gradient straight into it and return True; otherwise return False."""
    z = getattr(w, "_hds_zero", None)
    tgt = z.wgrad_target(w) if z is not None else None
    if tgt is None:
        return False
    g, fresh = tgt
    compute(g, not fresh)
    z.wgrad_written(w)
    return True


def grad_accumulator(w, dtype):
    """The ZeRO-owned gradient buffer of ``w`` to ADD a gradient contribution into directly (returning None to
    autograd instead of a dense tensor), or None. A buffer still marked fresh (an in-place GEMM target that has
    not been written this window) holds last window's values and is cleared first."""
    z = getattr(w, "_hds_zero", None)
    g = w.grad if z is not None else None
    if g is None or g.dtype != dtype or not g.is_contiguous() or not z.accumulate_ok(w):
        return None
    if getattr(w, "_hds_gfresh", False):
        g.zero_()
        w._hds_gfresh = False
    return g


_FWD_GEMM = __import__("os").environ.get("HDS_GEMM_FWD", "0") == "1"  # experiment: hand-written MFMA fwd GEMM


_FWD_SPLIT = __import__("os").environ.get("HDS_FWD_SPLIT", "auto")  # auto | off | on
_FWD_CHOICE = {}


def _col_split(n):
    """Output-column split of an N that is not a multiple of the 4096-wide tiles hipBLASLt runs best (the fused
    Llama-3 qkv projection, N = 6144 = 4096 + 2048), or None."""
    if n <= 4096 or n % 4096 == 0 or (n % 4096) % 256:
        return None
    return n - n % 4096


def _split_fwd(x2, weight, n1):
    """y[:, :n1] = x W[:n1]^T and y[:, n1:] = x W[n1:]^T as two GEMMs writing column slices of ONE output (row
    stride N: no concatenation copy)."""
    y = torch.empty(x2.shape[0], weight.shape[0], dtype=x2.dtype, device=x2.device)
    torch.mm(x2, weight[:n1].t(), out=y[:, :n1])
    torch.mm(x2, weight[n1:].t(), out=y[:, n1:])
    return y


def _time(fn):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1)


def _linear_fwd(x, weight, bias):
    if _FWD_GEMM and bias is None and x.is_cuda and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16:
        from ...ops.gemm import gemm_nt, gemm_nt_supported
        x2 = x.reshape(-1, x.shape[-1])
        if gemm_nt_supported(x2.shape[0], weight.shape[0], x2.shape[1]) and x2.is_contiguous():
            return gemm_nt(x2, weight).view(*x.shape[:-1], weight.shape[0])
    n1 = _col_split(weight.shape[0])
    if (n1 is not None and _FWD_SPLIT != "off" and bias is None and x.is_cuda and x.dtype == weight.dtype
            and x.is_contiguous() and weight.is_contiguous()):
        x2 = x.reshape(-1, x.shape[-1])
        key = (x2.shape[0], weight.shape[0], x2.shape[1], x.dtype)
        split = _FWD_CHOICE.get(key) if _FWD_SPLIT == "auto" else True
        if split is None:  # timed once per shape: the split wins where hipBLASLt's pick for the odd N is slow
            t_fused = _time(lambda: F.linear(x2, weight))
            t_split = _time(lambda: _split_fwd(x2, weight, n1))
            split = _FWD_CHOICE[key] = t_split < 0.97 * t_fused
        if split:
            return _split_fwd(x2, weight, n1).view(*x.shape[:-1], weight.shape[0])
    return F.linear(x, weight, bias)


class LinearFunctionForZeroStage3(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, weight, bias=None):
        # a producer that also wrote x's transpose ([K, tokens], ops/activations.glu transposed=True) lets the
        # weight gradient run hipBLASLt's NT form without transposing x in the backward: save that copy, not x
        xt = getattr(x, "_hds_t", None)
        ctx.x_t = (xt is not None and xt.dim() == 2 and xt.shape[0] == x.shape[-1] and xt.dtype == x.dtype
                   and xt.shape[1] * xt.shape[0] == x.numel())
        ctx.save_for_backward(xt if ctx.x_t else x)
        ctx.weight = weight
        ctx.has_bias = bias is not None
        out = _linear_fwd(x, weight, bias)
        from ...offload import act_plan
        if act_plan.tracking() and not ctx.x_t:  # recomputable from its (saved) input: offload/act_plan.py
            act_plan.tag(out, "linear_out", fn=_linear_fwd, srcs=(x, weight, bias))
        return out

    @staticmethod
    def backward(ctx, dy):
        (x, ) = ctx.saved_tensors
        xt = None
        if ctx.x_t:
            xt, x = x, None
        dyt = getattr(dy, "_hds_t", None)  # the output gradient's transpose, when its producer wrote one
        if dyt is not None and (dyt.dim() != 2 or dyt.shape[0] != dy.shape[-1] or dyt.dtype != dy.dtype):
            dyt = None
        w = ctx.weight
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if dy.is_cuda and dy.dim() >= 2 and w.dtype == dy.dtype:
                from ...ops.gemm import dgrad
                dx = dgrad(dy.reshape(-1, dy.shape[-1]), w).view(*dy.shape[:-1], w.shape[1])
            else:
                dx = dy.matmul(w.to(dy.dtype))
        if ctx.needs_input_grad[1]:
            dy2 = dy.reshape(-1, dy.shape[-1])
            x2 = x.reshape(-1, x.shape[-1]).to(dy.dtype) if x is not None else None
            xt2 = xt.to(dy.dtype) if xt is not None else None

            def gemm(out, accumulate):
                from ...ops.gemm import wgrad
                wgrad(dy2, x2, out, accumulate, dyt=dyt, xt=xt2)

            if not write_weight_grad(w, gemm):
                dw = dy2.t().matmul(x2) if x2 is not None else dy2.t().matmul(xt2.t())
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).sum(0)
        return dx, dw, db


def zero3_linear(x, weight, bias=None):
    return LinearFunctionForZeroStage3.apply(x, weight, bias)


def _mel_forward(self, x):
    return zero3_linear(x, self.weight, self.bias)


def wrap_memory_efficient_linears(module, only=None):
    """Route every nn.Linear under ``module`` (or those whose weight id is in ``only``) through the Function
    (instance-level forward override)."""
    n = 0
    for m in module.modules():
        if isinstance(m, nn.Linear) and not getattr(m, "_hds_mel", False) and \
                (only is None or id(m.weight) in only):
            m.forward = types.MethodType(_mel_forward, m)
            m._hds_mel = True
            n += 1
    return n
