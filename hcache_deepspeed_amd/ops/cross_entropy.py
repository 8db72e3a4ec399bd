"""Cross-entropy kernels: plain (over given logits) and fused LM-head + CE (chunked, grads eager).

The reference has no fused loss; HF Llama materialises [T, V] fp32 logits (8 GB for 8k tokens at
V=128256). Here :func:`fused_linear_cross_entropy` runs the LM-head GEMM in row chunks; for each
chunk the HIP kernel (csrc/kernels/xent.hip) computes loss + LSE and overwrites the logits with
d(loss)/d(logits), then two GEMMs produce d(hidden) for the chunk and accumulate d(W) in fp32.
The backward only scales those by the incoming grad -- the logits are never stored and never
recomputed.
"""
import torch
import torch.nn.functional as F

from . import native


def _xent_native(logits, target, ignore_index, grad_scale, write_grad, label_smoothing=0.0):
    rows, V = logits.shape
    loss = torch.empty(rows, device=logits.device, dtype=torch.float32)
    lse = torch.empty(rows, device=logits.device, dtype=torch.float32)
    native.check(
        native.kernels().hds_xent(native.dt(logits), logits.data_ptr(), target.data_ptr(), loss.data_ptr(),
                                  lse.data_ptr(), rows, V, logits.stride(0), int(ignore_index), float(grad_scale),
                                  int(write_grad), float(label_smoothing), native.stream()), "xent")
    return loss, lse


class _CEFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, logits, target, ignore_index, label_smoothing):
        l2 = logits.reshape(-1, logits.shape[-1])
        t = target.reshape(-1).to(torch.int64).contiguous()
        if native.use_native(l2):
            buf = l2.contiguous().clone() if logits.requires_grad else l2.contiguous()
            loss, _ = _xent_native(buf, t, ignore_index, 1.0, int(logits.requires_grad), label_smoothing)
            ctx.save_for_backward(buf if logits.requires_grad else None)
        else:
            lf = l2.float()
            loss = F.cross_entropy(lf, t, ignore_index=ignore_index, reduction="none",
                                   label_smoothing=label_smoothing)
            ctx.save_for_backward(lf)
        ctx.t = t
        ctx.args = (ignore_index, label_smoothing, logits.shape, logits.dtype)
        return loss.view(target.shape)

    @staticmethod
    def backward(ctx, dloss):
        (buf, ) = ctx.saved_tensors
        ignore_index, ls, shape, dtype = ctx.args
        d = dloss.reshape(-1, 1).float()
        if buf.dtype != torch.float32 or native.use_native(buf):
            g = (buf.float() * d).to(dtype)
        else:
            with torch.enable_grad():
                lf = buf.detach().requires_grad_(True)
                loss = F.cross_entropy(lf, ctx.t, ignore_index=ignore_index, reduction="none", label_smoothing=ls)
                (g, ) = torch.autograd.grad(loss, lf, d.view(-1))
            g = g.to(dtype)
        return g.view(shape), None, None, None


def cross_entropy(logits, target, ignore_index=-100, reduction="mean", label_smoothing=0.0):
    loss = _CEFn.apply(logits, target, ignore_index, label_smoothing)
    if reduction == "none":
        return loss
    if reduction == "sum":
        return loss.sum()
    valid = (target != ignore_index).sum().clamp(min=1)
    return loss.sum() / valid


def _mm_f32(a, b):
    """a @ b with fp32 output (bf16 inputs on GPU keep fp32 accumulation in the output)."""
    if a.is_cuda:
        return torch.mm(a, b, out_dtype=torch.float32)
    return torch.mm(a.float(), b.float())


_ADDMM_OUT_DTYPE = [None]  # None = not probed yet


def _probe_addmm_out_dtype(device):
    """One tiny probe: does this torch build accept ``addmm(..., out_dtype=float32)`` on bf16 inputs? Only the
    capability probe may fail; real errors (OOM, HIP faults) in the hot path propagate."""
    try:
        a = torch.zeros(2, 2, dtype=torch.bfloat16, device=device)
        acc = torch.zeros(2, 2, dtype=torch.float32, device=device)
        torch.addmm(acc, a, a, out_dtype=torch.float32, out=acc)
        _ADDMM_OUT_DTYPE[0] = True
    except (TypeError, RuntimeError) as e:
        from ..utils.logging import logger
        logger.warning(f"fused linear CE: addmm(out_dtype=fp32) unsupported ({e}); using mm + add")
        _ADDMM_OUT_DTYPE[0] = False
    return _ADDMM_OUT_DTYPE[0]


def _addmm_f32_(acc, a, b):
    """acc += a @ b with bf16 inputs and the fp32 accumulator folded into the GEMM (hipBLASLt beta=1): saves
    one full fp32 read+write of the [V, H] LM-head gradient per chunk (7 x 1.07 ms per step at the bench
    shape, profiles/rocprof_kernel_stats_r1_final.csv)."""
    if acc.is_cuda:
        ok = _ADDMM_OUT_DTYPE[0]
        if ok is None:
            ok = _probe_addmm_out_dtype(acc.device)
        if ok:
            torch.addmm(acc, a, b, out_dtype=torch.float32, out=acc)
            return
    acc.add_(_mm_f32(a, b))


class _FusedLinearCEFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, hidden, weight, target, ignore_index, chunk_rows, label_smoothing):
        T, H = hidden.shape
        V = weight.shape[0]
        need_grad = hidden.requires_grad or weight.requires_grad
        t = target.reshape(-1).to(torch.int64).contiguous()
        losses = torch.empty(T, device=hidden.device, dtype=torch.float32)
        dh = torch.empty_like(hidden) if (need_grad and hidden.requires_grad) else None
        want_dw = need_grad and weight.requires_grad
        dw = None  # fp32 accumulator: the first chunk's GEMM writes it (beta = 0), no zero-fill pass
        native_path = native.use_native(hidden)
        wcache = {}  # the LM-head weight transposed once for every chunk's dgrad (NT layout)
        for s in range(0, T, chunk_rows):
            e = min(T, s + chunk_rows)
            hc = hidden[s:e]
            logits = torch.mm(hc, weight.t())  # [rows, V] in activation dtype
            if native_path:
                loss_c, _ = _xent_native(logits, t[s:e], ignore_index, 1.0, int(need_grad), label_smoothing)
                dl = logits
            else:
                lf = logits.float().requires_grad_(need_grad)
                with torch.enable_grad():
                    loss_c = F.cross_entropy(lf, t[s:e], ignore_index=ignore_index, reduction="none",
                                             label_smoothing=label_smoothing)
                    if need_grad:
                        (dl, ) = torch.autograd.grad(loss_c.sum(), lf)
                        dl = dl.to(hidden.dtype)
                loss_c = loss_c.detach()
            losses[s:e] = loss_c
            if need_grad:
                if dh is not None:
                    if dl.is_cuda:
                        from .gemm import dgrad
                        dgrad(dl, weight, out=dh[s:e], cache=wcache)
                    else:
                        torch.mm(dl, weight, out=dh[s:e])
                if want_dw:
                    if dl.is_cuda and _ADDMM_OUT_DTYPE[0] is not False and (
                            _ADDMM_OUT_DTYPE[0] or _probe_addmm_out_dtype(dl.device)):
                        from .gemm import wgrad  # fp32 accumulator, layout chosen per shape (TN or NT)
                        if dw is None:
                            dw = torch.empty(V, H, device=hidden.device, dtype=torch.float32)
                        wgrad(dl, hc, dw, accumulate=s > 0)
                    elif dw is None:
                        dw = _mm_f32(dl.t(), hc)
                    else:
                        _addmm_f32_(dw, dl.t(), hc)
            del logits
        del wcache
        ctx.save_for_backward(dh, dw)
        ctx.wdtype = weight.dtype
        ctx.weight = weight  # the Parameter object: its gradient may be written in place (ZeRO)
        ctx.mark_non_differentiable(losses)
        return losses.sum(), losses

    @staticmethod
    def backward(ctx, dsum, _dlosses):
        # the loss is returned already summed, so the upstream gradient is one scalar that scales
        # the eagerly computed d(hidden) and d(W)
        dh, dw = ctx.saved_tensors
        gh = (dh * dsum.to(dh.dtype)) if dh is not None else None
        gw = None
        if dw is not None:
            dw.mul_(dsum.float())
            from ..runtime.zero.linear import write_weight_grad

            def put(out, accumulate):  # fp32 accumulator -> the bf16 gradient buffer (one pass)
                out.add_(dw) if accumulate else out.copy_(dw)

            if not write_weight_grad(ctx.weight, put):
                gw = dw.to(ctx.wdtype)
        return gh, gw, None, None, None, None


def fused_linear_cross_entropy(hidden, weight, target, ignore_index=-100, reduction="mean", chunk_rows=4096,
                               label_smoothing=0.0):
    """loss(hidden @ weight.T, target) without materialising the logits. hidden: [T, H], weight: [V, H]."""
    h2 = hidden.reshape(-1, hidden.shape[-1])
    if reduction == "none":
        return cross_entropy(torch.mm(h2, weight.t()), target.reshape(-1), ignore_index, "none", label_smoothing)
    total, _ = _FusedLinearCEFn.apply(h2, weight, target, ignore_index, int(chunk_rows), float(label_smoothing))
    if reduction == "sum":
        return total
    valid = (target.reshape(-1) != ignore_index).sum().clamp(min=1)
    return total / valid
