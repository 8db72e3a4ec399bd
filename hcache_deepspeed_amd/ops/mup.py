"""muP optimizers: ``MuAdam``, ``MuAdamW``, ``MuSGD``.

Reference parity: the reference engine accepts ``"optimizer": {"type": "MuAdam" | "MuAdamW" | "MuSGD"}`` and builds
them from the external ``mup`` package (runtime/engine.py:1503-1523). ``mup`` is not installed here, so the width
rules of Maximal Update Parametrization (Yang et al., Tensor Programs V) are implemented directly:

* Adam: matrix-like parameters (two infinite dims: hidden x hidden) get ``lr / width_mult``; vector-like
  (one infinite dim: embeddings, biases, norms, readout) and scalar-like keep ``lr``. Without decoupled weight
  decay the L2 coefficient is multiplied by ``width_mult`` so ``lr * wd`` is width-invariant.
* SGD: vector-like parameters get ``lr * width_mult``; matrix-like get ``lr * fanout_mult / fanin_mult``.

The width information is read, in order, from a mup-style ``p.infshape`` (duck-typed: ``ninf()``,
``width_mult()``, and ``[i].width_mult()`` for SGD), or from the attributes ``p.mup_width_mult`` (float) and
``p.mup_ninf`` (0/1/2; default 2 for ``p.dim() >= 2`` else 1), set by :func:`set_base_shapes`.

The multiplier is stored as the group key ``lr_mult`` and applied at update time by the fused HIP optimizers and
the ZeRO flat-shard step (``lr`` itself stays unscaled), so LR schedulers that write ``group["lr"]`` keep the muP
ratios — the reference/mup approach of pre-scaling ``lr`` at construction loses them on the first scheduler step.
"""
from collections import defaultdict

import torch

from .optimizers import FusedAdam


def _width_info(p):
    inf = getattr(p, "infshape", None)
    if inf is not None:
        return int(inf.ninf()), float(inf.width_mult()), inf
    wm = getattr(p, "mup_width_mult", None)
    if wm is None:
        return 0, 1.0, None
    ninf = getattr(p, "mup_ninf", 2 if p.dim() >= 2 else 1)
    return int(ninf), float(wm), None


def set_base_shapes(model, base_model):
    """Give every parameter of ``model`` its muP width multiplier relative to the same-named parameter of
    ``base_model`` (a narrower copy of the architecture): ``width_mult = fan_in / base_fan_in`` on the last
    dim, and ``mup_ninf`` = number of dims that grew. Mirrors ``mup.set_base_shapes`` for the optimizer rules."""
    base = dict(base_model.named_parameters())
    for name, p in model.named_parameters():
        b = base.get(name)
        if b is None or b.dim() != p.dim():
            continue
        grown = [i for i in range(p.dim()) if p.shape[i] != b.shape[i]]
        p.mup_ninf = len(grown)
        fan_dim = p.dim() - 1 if (p.dim() - 1) in grown else (grown[0] if grown else p.dim() - 1)
        p.mup_width_mult = p.shape[fan_dim] / b.shape[fan_dim]
        if p.dim() >= 2:
            p.mup_fanout_mult = p.shape[0] / b.shape[0]
            p.mup_fanin_mult = p.shape[-1] / b.shape[-1]
    return model


def _split_groups(params, defaults, rule):
    groups = list(params)
    if groups and not isinstance(groups[0], dict):
        groups = [{"params": groups}]
    out = []
    for g in groups:
        if "lr_mult" in g:  # already split (e.g. re-created by the ZeRO generic path)
            out.append(g)
            continue
        buckets = defaultdict(list)
        for p in g["params"]:
            buckets[rule(p)].append(p)
        for (lr_mult, wd_mult), ps in buckets.items():
            ng = {k: v for k, v in g.items() if k != "params"}
            ng["params"] = ps
            ng["lr_mult"] = lr_mult
            if wd_mult != 1.0:
                ng["weight_decay"] = ng.get("weight_decay", defaults.get("weight_decay", 0.0)) * wd_mult
            out.append(ng)
    return out


def _adam_rule(decoupled_wd):

    def rule(p):
        ninf, wm, _ = _width_info(p)
        if ninf == 2:
            return 1.0 / wm, (1.0 if decoupled_wd else wm)
        return 1.0, 1.0

    return rule


class MuAdam(FusedAdam):
    """Adam with muP learning-rate scaling over the fused HIP Adam kernel (L2 weight decay)."""

    _decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, **kw):
        kw.pop("adam_w_mode", None)
        groups = _split_groups(params, dict(weight_decay=weight_decay), _adam_rule(self._decoupled))
        super().__init__(groups, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                         adam_w_mode=self._decoupled, **kw)


class MuAdamW(MuAdam):
    """AdamW (decoupled weight decay) with muP learning-rate scaling."""

    _decoupled = True


def _sgd_rule(p):
    ninf, wm, inf = _width_info(p)
    if ninf == 1:
        return wm, 1.0 / wm
    if ninf == 2:
        if inf is not None:
            r = float(inf[0].width_mult()) / float(inf[1].width_mult())
        else:
            r = getattr(p, "mup_fanout_mult", 1.0) / getattr(p, "mup_fanin_mult", wm)
        return r, 1.0 / r
    return 1.0, 1.0


class MuSGD(torch.optim.SGD):
    """SGD with muP learning-rate scaling (``lr_mult`` applied for the duration of each step)."""

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, **kw):
        groups = _split_groups(params, dict(weight_decay=weight_decay), _sgd_rule)
        super().__init__(groups, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                         nesterov=nesterov, **kw)

    @torch.no_grad()
    def step(self, closure=None):
        saved = [g["lr"] for g in self.param_groups]
        for g in self.param_groups:
            g["lr"] = g["lr"] * g.get("lr_mult", 1.0)
        try:
            return super().step(closure)
        finally:
            for g, lr in zip(self.param_groups, saved):
                g["lr"] = lr
