"""RMSNorm / LayerNorm (+ fused residual add) with HIP forward and backward.

Reference parity: inference kernels ``rms_norm``/``pre_rms_norm``/``fused_ln``/``fused_residual_ln``
(deepspeed/inference/v2/kernels/core_ops/cuda_rms_norm/rms_norm.py, cuda_layer_norm/*.py) and the
training LayerNorm of csrc/transformer/normalize_kernels.cu. The kernels are in
csrc/kernels/norm.hip; CPU tensors run the fp32 torch reference below.
"""
import torch
import torch.nn as nn

from . import native
from ..offload import act_plan as _ap


def _ref_norm(x, residual, weight, bias, eps, is_ln):
    h = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    hf = h.float()
    if is_ln:
        mean = hf.mean(-1, keepdim=True)
        var = ((hf - mean) ** 2).mean(-1, keepdim=True)
    else:
        mean = torch.zeros_like(hf[..., :1])
        var = (hf * hf).mean(-1, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    y = (hf - mean) * rstd * weight.float()
    if bias is not None:
        y = y + bias.float()
    return y.to(x.dtype), h


def _native_fwd(x2, r2, weight, bias, eps, is_ln):
    rows, cols = x2.shape
    y = torch.empty_like(x2)
    h = torch.empty_like(x2) if r2 is not None else None
    rstd = torch.empty(rows, device=x2.device, dtype=torch.float32)
    mean = torch.empty(rows, device=x2.device, dtype=torch.float32) if is_ln else None
    if rows:
        lib = native.kernels()
        native.check(
            lib.hds_norm_fwd(int(is_ln), native.dt(x2), native.dt(weight), x2.data_ptr(), native.ptr(r2),
                             native.ptr(h), weight.data_ptr(), native.ptr(bias), y.data_ptr(), native.ptr(mean),
                             rstd.data_ptr(), rows, cols, float(eps), native.stream()), "norm_fwd")
    return y, (h if h is not None else x2), mean, rstd


def _native_bwd(dy2, h2, dres2, weight, bias, mean, rstd, is_ln, need_wgrad):
    rows, cols = h2.shape
    dx = torch.empty_like(h2)
    lib = native.kernels()
    nparts = lib.hds_norm_bwd_nparts(rows)
    dw_part = torch.empty(nparts, cols, device=h2.device, dtype=torch.float32)
    db_part = torch.empty(nparts, cols, device=h2.device, dtype=torch.float32) if is_ln else None
    dw = torch.empty_like(weight) if need_wgrad else None
    db = torch.empty_like(bias) if (bias is not None and need_wgrad) else None
    if rows:
        native.check(
            lib.hds_norm_bwd(int(is_ln), native.dt(h2), native.dt(weight), dy2.data_ptr(), h2.data_ptr(),
                             native.ptr(dres2), weight.data_ptr(), native.ptr(mean), rstd.data_ptr(), dx.data_ptr(),
                             dw_part.data_ptr(), native.ptr(db_part), nparts, native.ptr(dw), native.ptr(db), 0, rows,
                             cols, native.stream()), "norm_bwd")
    else:
        if dw is not None:
            dw.zero_()
        if db is not None:
            db.zero_()
    return dx, dw, db


def _norm_out(h, weight, bias, eps, is_ln):
    """Recompute the norm output from the saved pre-norm sum (bit-identical: the fused kernel rounds the sum to the
    activation dtype before its statistics, like this unfused call)."""
    if native.use_native(h):
        return _native_fwd(h.contiguous(), None, weight, bias, eps, is_ln)[0]
    return _ref_norm(h, None, weight, bias, eps, is_ln)[0]


class _NormFn(torch.autograd.Function):
    """y = norm(x [+ residual]); returns (y, h) where h is the pre-norm sum (the new residual)."""

    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, is_ln):
        shape = x.shape
        H = shape[-1]
        x2 = x.reshape(-1, H)
        r2 = residual.reshape(-1, H) if residual is not None else None
        if native.use_native(x2):
            x2 = x2.contiguous()
            r2 = r2.contiguous() if r2 is not None else None
            y, h, mean, rstd = _native_fwd(x2, r2, weight, bias, eps, is_ln)
        else:
            y, h = _ref_norm(x2, r2, weight, bias, eps, is_ln)
            hf = h.float()
            mean = hf.mean(-1) if is_ln else None
            var = ((hf - (mean[:, None] if is_ln else 0.0)) ** 2).mean(-1)
            rstd = torch.rsqrt(var + eps)
        if _ap.tracking():  # per-tensor activation plan: the output (and the new residual) can be recomputed
            if r2 is not None:
                _ap.tag(h, "resid", fn=torch.add, srcs=(x2, r2))
            _ap.tag(y, "norm_out", fn=_norm_out, srcs=(h, weight, bias, float(eps), bool(is_ln)))
        ctx.save_for_backward(h, weight, bias, mean, rstd)
        ctx.is_ln = is_ln
        ctx.has_res = residual is not None
        ctx.shape = shape
        return y.view(shape), h.view(shape)

    @staticmethod
    def backward(ctx, dy, dh):
        h, weight, bias, mean, rstd = ctx.saved_tensors
        H = ctx.shape[-1]
        dy2 = dy.reshape(-1, H)
        dres = dh.reshape(-1, H) if (dh is not None and ctx.has_res) else None
        need_w = ctx.needs_input_grad[2]
        if native.use_native(h):
            dx, dw, db = _native_bwd(dy2.contiguous(), h, dres.contiguous() if dres is not None else None, weight,
                                     bias, mean, rstd, ctx.is_ln, need_w)
        else:
            hf = h.float()
            xh = (hf - (mean[:, None] if ctx.is_ln else 0.0)) * rstd[:, None]
            g = dy2.float() * weight.float()
            dx = rstd[:, None] * (g - xh * (g * xh).mean(-1, keepdim=True) -
                                  (g.mean(-1, keepdim=True) if ctx.is_ln else 0.0))
            if dres is not None:
                dx = dx + dres.float()
            dx = dx.to(h.dtype)
            dw = (dy2.float() * xh).sum(0).to(weight.dtype)
            db = dy2.float().sum(0).to(bias.dtype) if bias is not None else None
        dx = dx.view(ctx.shape)
        dres_out = dx if ctx.has_res else None
        return dx, dres_out, dw, db, None, None


def rms_norm(x, weight, eps=1e-6, residual=None):
    """Returns y, or (y, new_residual) when ``residual`` is given (fused add + norm)."""
    y, h = _NormFn.apply(x, residual, weight, None, eps, False)
    return (y, h) if residual is not None else y


def layer_norm(x, weight, bias=None, eps=1e-5, residual=None):
    y, h = _NormFn.apply(x, residual, weight, bias, eps, True)
    return (y, h) if residual is not None else y


class RMSNorm(nn.Module):

    def __init__(self, hidden_size, eps=1e-6, dtype=None, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size, dtype=dtype, device=device))
        self.eps = eps

    def reset_parameters(self):
        with torch.no_grad():
            self.weight.fill_(1.0)

    def forward(self, x, residual=None):
        return rms_norm(x, self.weight, self.eps, residual)


class LayerNorm(nn.Module):

    def __init__(self, hidden_size, eps=1e-5, bias=True, dtype=None, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size, dtype=dtype, device=device))
        self.bias = nn.Parameter(torch.zeros(hidden_size, dtype=dtype, device=device)) if bias else None
        self.eps = eps

    def reset_parameters(self):
        with torch.no_grad():
            self.weight.fill_(1.0)
            if self.bias is not None:
                self.bias.zero_()

    def forward(self, x, residual=None):
        return layer_norm(x, self.weight, self.bias, self.eps, residual)
