"""Fused GPU optimizers (Adam/AdamW, Lion, LAMB, Adagrad) over HIP kernels (csrc/kernels/optim.hip).

Reference parity: ``FusedAdam`` (deepspeed/ops/adam/fused_adam.py:18), ``FusedLion``
(ops/lion/fused_lion.py:17), ``FusedLamb`` (ops/lamb/fused_lamb.py:14) -- same constructor
arguments and ``step()`` semantics, so user code / configs keep working.

Two levels:

* ``*_flat(...)`` functional updates of ONE flat partition -- what the ZeRO optimizers call (their
  fp32 master/moments are flat buffers). The bf16 working copy is written in the same pass, and the
  grad scale (loss-scale unscale x clip coefficient) can be a device scalar, so the step never syncs.
* ``torch.optim.Optimizer`` subclasses for arbitrary parameter lists, driven by a device-resident
  multi-tensor chunk table (one launch for any number of tensors).
"""
import math

import torch

from . import native


def _glr(group):
    """Effective learning rate of a param group: ``lr`` times the muP width multiplier ``lr_mult`` (ops/mup.py);
    schedulers keep writing the unscaled ``lr``."""
    return group["lr"] * group.get("lr_mult", 1.0)


def _f(x):
    return float(x)


# ------------------------------------------------------------------------------------------
# flat functional forms
# ------------------------------------------------------------------------------------------
def _native_lp(p, lp_out):
    """The flat kernels write their low-precision copy of the updated parameters as bf16: hand them only a bf16
    target. Any other ``lp_out`` (fp32 training's compute copy, fp16) is refreshed from ``p`` after the kernel --
    unless it IS ``p``. Returns (kernel target, tensor to copy into afterwards)."""
    if lp_out is None or lp_out.dtype == torch.bfloat16:
        return lp_out, None
    if lp_out.dtype == p.dtype and lp_out.data_ptr() == p.data_ptr():
        return None, None
    return None, lp_out


def adam_flat(p, g, m, v, step, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=True, bias_correction=True,
              lp_out=None, grad_scale=1.0, dev_scale=None, found_inf=None):
    b1, b2 = betas
    bc1 = 1 - b1**step if bias_correction else 1.0
    bc2 = 1 - b2**step if bias_correction else 1.0
    if native.use_native(p):
        lp, after = _native_lp(p, lp_out)
        native.check(
            native.kernels().hds_adam_flat(native.dt(p), native.dt(g), p.data_ptr(), g.data_ptr(), m.data_ptr(),
                                           v.data_ptr(), native.ptr(lp), p.numel(), _f(lr), _f(b1), _f(b2),
                                           _f(eps), _f(weight_decay), _f(bc1), _f(bc2), int(adamw), _f(grad_scale),
                                           native.ptr(dev_scale), native.ptr(found_inf), native.stream()),
            "adam_flat")
        if after is not None:
            after.copy_(p)
        return
    if found_inf is not None and bool(found_inf.item()):
        return
    sc = grad_scale * (dev_scale.item() if dev_scale is not None else 1.0)
    pf = p.float()
    gf = g.float() * sc
    if not adamw and weight_decay:
        gf = gf + weight_decay * pf
    m.mul_(b1).add_(gf, alpha=1 - b1)
    v.mul_(b2).addcmul_(gf, gf, value=1 - b2)
    upd = (m / bc1) / ((v / bc2).sqrt() + eps)
    if adamw and weight_decay:
        upd = upd + weight_decay * pf
    pf = pf - lr * upd
    p.copy_(pf)
    if lp_out is not None:
        lp_out.copy_(pf)


def lion_flat(p, g, m, lr, betas=(0.9, 0.99), weight_decay=0.0, lp_out=None, grad_scale=1.0, dev_scale=None,
              found_inf=None):
    b1, b2 = betas
    if native.use_native(p):
        lp, after = _native_lp(p, lp_out)
        native.check(
            native.kernels().hds_lion_flat(native.dt(p), native.dt(g), p.data_ptr(), g.data_ptr(), m.data_ptr(),
                                           native.ptr(lp), p.numel(), _f(lr), _f(b1), _f(b2), _f(weight_decay),
                                           _f(grad_scale), native.ptr(dev_scale), native.ptr(found_inf),
                                           native.stream()), "lion_flat")
        if after is not None:
            after.copy_(p)
        return
    if found_inf is not None and bool(found_inf.item()):
        return
    sc = grad_scale * (dev_scale.item() if dev_scale is not None else 1.0)
    gf = g.float() * sc
    pf = p.float()
    c = b1 * m + (1 - b1) * gf
    pf = pf * (1 - lr * weight_decay) - lr * torch.sign(c)
    m.mul_(b2).add_(gf, alpha=1 - b2)
    p.copy_(pf)
    if lp_out is not None:
        lp_out.copy_(pf)


def adagrad_flat(p, g, s, lr, eps=1e-10, weight_decay=0.0, lp_out=None, grad_scale=1.0, dev_scale=None,
                 found_inf=None):
    if native.use_native(p):
        lp, after = _native_lp(p, lp_out)
        native.check(
            native.kernels().hds_adagrad_flat(native.dt(p), native.dt(g), p.data_ptr(), g.data_ptr(), s.data_ptr(),
                                              native.ptr(lp), p.numel(), _f(lr), _f(eps), _f(weight_decay),
                                              _f(grad_scale), native.ptr(dev_scale), native.ptr(found_inf),
                                              native.stream()), "adagrad_flat")
        if after is not None:
            after.copy_(p)
        return
    sc = grad_scale * (dev_scale.item() if dev_scale is not None else 1.0)
    pf = p.float()
    gf = g.float() * sc + weight_decay * pf
    s.addcmul_(gf, gf)
    pf = pf - lr * gf / (s.sqrt() + eps)
    p.copy_(pf)
    if lp_out is not None:
        lp_out.copy_(pf)


def grad_sumsq(tensors, out=None, found_inf=None):
    """Sum of squares of many tensors into a device fp32 scalar (+ non-finite flag), no host sync."""
    dev = tensors[0].device
    out = out if out is not None else torch.zeros(1, device=dev, dtype=torch.float32)
    if native.use_native(tensors[0]):
        lib = native.kernels()
        st = native.stream()
        for t in tensors:
            if t.numel() == 0:
                continue
            t = t if t.is_contiguous() else t.contiguous()
            native.check(lib.hds_sumsq(native.dt(t), t.data_ptr(), t.numel(), out.data_ptr(), native.ptr(found_inf),
                                       st), "sumsq")
        return out
    for t in tensors:
        tf = t.float()
        out.add_((tf * tf).sum())
        if found_inf is not None and not torch.isfinite(tf).all():
            found_inf.fill_(1)
    return out


def clip_coef(sumsq, max_norm, inv_scale=1.0, coef=None, norm_out=None):
    """coef = inv_scale * min(1, max_norm / (||g|| * inv_scale + 1e-6)) as a device scalar."""
    coef = coef if coef is not None else torch.empty(1, device=sumsq.device, dtype=torch.float32)
    if native.use_native(sumsq):
        native.check(native.kernels().hds_clip_coef(sumsq.data_ptr(), _f(max_norm), _f(inv_scale), coef.data_ptr(),
                                                    native.ptr(norm_out), native.stream()), "clip_coef")
        return coef
    nrm = sumsq.sqrt() * inv_scale
    if norm_out is not None:
        norm_out.copy_(nrm)
    c = torch.full_like(coef, inv_scale)
    if max_norm > 0:
        k = max_norm / (nrm + 1e-6)
        c = torch.where(k < 1, c * k, c)
    coef.copy_(c)
    return coef


# ------------------------------------------------------------------------------------------
# multi-tensor chunk tables
# ------------------------------------------------------------------------------------------
class _ChunkTable:
    """Device table {p, g, m, v, lp, numel} x N + chunk list, rebuilt only when pointers change."""

    def __init__(self):
        self.key = None
        self.tensors = None
        self.chunks = None
        self.nchunks = 0

    def get(self, rows, device):
        key = tuple(rows)
        if key != self.key:
            chunk = native.kernels().hds_multi_chunk_size()
            ch = []
            for i, r in enumerate(rows):
                n = r[5]
                for s in range(0, n, chunk):
                    ch.append((i, s))
            self.tensors = torch.tensor(rows, dtype=torch.int64).to(device, non_blocking=True)
            self.chunks = torch.tensor(ch if ch else [(0, 0)], dtype=torch.int64).to(device, non_blocking=True)
            self.nchunks = len(ch)
            self.key = key
        return self.tensors, self.chunks, self.nchunks


class FusedAdam(torch.optim.Optimizer):
    """Adam/AdamW with the reference FusedAdam signature (ops/adam/fused_adam.py:18)."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, adam_w_mode=True,
                 weight_decay=0.0, amsgrad=False, set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none
        self._tables = {}

    def zero_grad(self, set_to_none=True):
        super().zero_grad(set_to_none=self.set_grad_none or set_to_none)

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0, dev_scale=None, found_inf=None):
        loss = closure() if closure is not None else None
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            if "step" not in group:
                group["step"] = 0
            group["step"] += 1
            step = group["step"]
            bc1 = 1 - b1**step if group["bias_correction"] else 1.0
            bc2 = 1 - b2**step if group["bias_correction"] else 1.0
            buckets = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                st["step"] = step
                if not native.use_native(p):
                    adam_flat(p.data, p.grad, st["exp_avg"], st["exp_avg_sq"], step, _glr(group), (b1, b2),
                              group["eps"], group["weight_decay"], bool(self.adam_w_mode), group["bias_correction"],
                              grad_scale=grad_scale, dev_scale=dev_scale, found_inf=found_inf)
                    continue
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                buckets.setdefault((p.dtype, g.dtype), []).append(
                    (p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), 0, p.numel()))
            for (pd, gd), rows in buckets.items():
                tab = self._tables.setdefault((gi, pd, gd), _ChunkTable())
                tensors, chunks, n = tab.get(rows, group["params"][0].device)
                native.check(
                    native.kernels().hds_adam_multi(native.dt(pd), native.dt(gd), tensors.data_ptr(), chunks.data_ptr(),
                                                    n, _f(_glr(group)), _f(b1), _f(b2), _f(group["eps"]),
                                                    _f(group["weight_decay"]), _f(bc1), _f(bc2), self.adam_w_mode,
                                                    _f(grad_scale), native.ptr(dev_scale), native.ptr(found_inf),
                                                    native.stream()), "adam_multi")
        return loss


class FusedLion(torch.optim.Optimizer):
    """Lion (reference ops/lion/fused_lion.py:17)."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.99), weight_decay=0.0, set_grad_none=True):
        super().__init__(params, dict(lr=lr, betas=betas, weight_decay=weight_decay))
        self.set_grad_none = set_grad_none

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0, dev_scale=None, found_inf=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                g = p.grad.contiguous()
                lion_flat(p.data, g, st["exp_avg"], _glr(group), group["betas"], group["weight_decay"],
                          grad_scale=grad_scale, dev_scale=dev_scale, found_inf=found_inf)
        return loss


class FusedLamb(torch.optim.Optimizer):
    """LAMB with per-tensor trust ratio (reference ops/lamb/fused_lamb.py:14)."""

    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, eps_inside_sqrt=False,
                 weight_decay=0.0, max_grad_norm=0.0, max_coeff=10.0, min_coeff=0.01, amsgrad=False):
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        max_coeff=max_coeff, min_coeff=min_coeff)
        super().__init__(params, defaults)
        self._tables = {}
        self.lamb_coeffs = []

    @torch.no_grad()
    def step(self, closure=None, grad_scale=1.0, dev_scale=None, found_inf=None):
        loss = closure() if closure is not None else None
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            group["step"] = group.get("step", 0) + 1
            step = group["step"]
            bc1 = 1 - b1**step if group["bias_correction"] else 1.0
            bc2 = 1 - b2**step if group["bias_correction"] else 1.0
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
            if native.use_native(params[0]):
                rows = [(p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                         self.state[p]["exp_avg_sq"].data_ptr(), 0, p.numel()) for p in params]
                pd, gd = params[0].dtype, params[0].grad.dtype
                tab = self._tables.setdefault(gi, _ChunkTable())
                tensors, chunks, n = tab.get(rows, params[0].device)
                norms = torch.zeros(2 * len(params), device=params[0].device, dtype=torch.float32)
                native.check(
                    native.kernels().hds_lamb_multi(native.dt(pd), native.dt(gd), tensors.data_ptr(),
                                                    chunks.data_ptr(), n, norms.data_ptr(), _f(_glr(group)), _f(b1),
                                                    _f(b2), _f(group["eps"]), _f(group["weight_decay"]), _f(bc1),
                                                    _f(bc2), _f(group["max_coeff"]), _f(group["min_coeff"]),
                                                    _f(grad_scale), native.ptr(dev_scale), native.ptr(found_inf),
                                                    native.stream()), "lamb_multi")
                continue
            for p in params:
                st = self.state[p]
                gf = p.grad.float() * grad_scale
                m, v = st["exp_avg"], st["exp_avg_sq"]
                m.mul_(b1).add_(gf, alpha=1 - b1)
                v.mul_(b2).addcmul_(gf, gf, value=1 - b2)
                pf = p.data.float()
                u = (m / bc1) / ((v / bc2).sqrt() + group["eps"]) + group["weight_decay"] * pf
                pn, un = pf.norm(), u.norm()
                trust = (pn / un) if (pn > 0 and un > 0) else torch.tensor(1.0)
                trust = float(min(max(float(trust), group["min_coeff"]), group["max_coeff"]))
                p.data.copy_(pf - _glr(group) * trust * u)
        return loss
