"""1-bit Adam, 0/1 Adam and 1-bit LAMB on the flat-shard (ZeRO-0) store.

Reference parity: runtime/fp16/onebit/adam.py (``OnebitAdam`` :14, warm-up then frozen variance with
compressed momentum all-reduce :238-300), zoadam.py (``ZeroOneAdam`` :14, variance updated on a growing
interval until ``var_freeze_step``), lamb.py (``OnebitLamb`` :15, frozen per-tensor LAMB coefficients with
bounded adaptive factors), engine.py :1476-1490 (incompatible with ZeRO >= 1).

Mechanics here: the optimizer classes only carry hyper-parameters; ``OnebitZeroOptimizer`` runs them
over the ZeRO-0 flat store. During warm-up gradients are bucket-all-reduced as in plain data
parallelism and the step is the fused Adam (or LAMB) kernel. Once compression starts, the gradient
all-reduce is skipped entirely (gradients stay local), each rank folds its own gradient into the
momentum, and the momentum -- one flat fp32 buffer -- goes through ONE error-compensated 1-bit
all-reduce (runtime/comm/compressed.py): 1/32 of the bytes of an fp32 all-reduce over xGMI.
"""
import math

import torch

from ..comm.compressed import compressed_allreduce, padded_size
from ..zero.optimizer import ZeroOptimizer


class _OnebitBase(torch.optim.Optimizer):
    """Hyper-parameter holder; the step runs inside OnebitZeroOptimizer (requires the engine)."""
    kind = "onebit_adam"

    def __init__(self, params, deepspeed=None, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0, amsgrad=False, cuda_aware=False,
                 comm_backend_name="nccl", **extra):
        if amsgrad:
            raise RuntimeError(f"{type(self).__name__} does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=tuple(betas), eps=eps,
                        weight_decay=weight_decay, max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.deepspeed = deepspeed
        self.eps_mode = 0 if eps_inside_sqrt else 1
        self.comm_backend_name = comm_backend_name
        for k, v in extra.items():
            setattr(self, k, v)

    def step(self, closure=None):
        raise RuntimeError(f"{type(self).__name__} runs through deepspeed.initialize (ZeRO stage 0)")


class OnebitAdam(_OnebitBase):
    kind = "onebit_adam"

    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, **kw):
        super().__init__(params, deepspeed, lr, freeze_step=int(freeze_step), **kw)


class ZeroOneAdam(_OnebitBase):
    kind = "zero_one_adam"

    def __init__(self, params, deepspeed=None, lr=1e-3, var_freeze_step=100000, var_update_scaler=16,
                 local_step_scaler=32678, local_step_clipper=16, **kw):
        super().__init__(params, deepspeed, lr, var_freeze_step=int(var_freeze_step),
                         var_update_scaler=int(var_update_scaler), local_step_scaler=int(local_step_scaler),
                         local_step_clipper=int(local_step_clipper), **kw)


class OnebitLamb(_OnebitBase):
    kind = "onebit_lamb"

    def __init__(self, params, deepspeed=None, lr=1e-3, freeze_step=100000, max_coeff=10.0, min_coeff=0.01,
                 coeff_beta=0.9, factor_max=4.0, factor_min=0.5, factor_threshold=0.1, **kw):
        super().__init__(params, deepspeed, lr, freeze_step=int(freeze_step), max_coeff=max_coeff,
                         min_coeff=min_coeff, coeff_beta=coeff_beta, factor_max=factor_max, factor_min=factor_min,
                         factor_threshold=factor_threshold, **kw)


def make_onebit(name, params, kw, engine):
    cls = {"onebitadam": OnebitAdam, "zerooneadam": ZeroOneAdam, "onebitlamb": OnebitLamb}[name]
    kw = dict(kw)
    return cls(params, deepspeed=engine, **kw)


class OnebitZeroOptimizer(ZeroOptimizer):
    """ZeRO-0 flat store + 1-bit compressed momentum synchronisation."""

    def __init__(self, init_optimizer, module, config, stage, **kw):
        assert int(stage) == 0, "1-bit optimizers are incompatible with ZeRO stages >= 1 (reference engine.py:1476)"
        super().__init__(init_optimizer, module, config, stage, **kw)
        self.ob = init_optimizer
        self.ob_kind = init_optimizer.kind
        self.n_steps = 0
        if self.ob_kind == "zero_one_adam":
            self.compressing = True  # 0/1 Adam compresses from the first step
            self.var_interval, self.var_counter, self.var_frozen = 1, 0, False
        else:
            self.compressing = False
        self._werr = self._serr = None
        if self.ob_kind == "onebit_lamb":
            self.lamb_coeff = {}      # per-parameter frozen LAMB coefficient
            self.lamb_last = {}

    # gradients stay local once compression is on
    def _reduce_unit(self, u):
        if self.compressing:
            if not u.direct:
                self.store.grad_slice(u).copy_(u.grad_full)
            return
        super()._reduce_unit(u)

    def _param_views(self, buf):
        for u in self.units:
            base = buf[u.store_off:u.store_off + u.shard]
            for i, p in enumerate(u.params):
                yield p, u.param_view(base, i)

    def _alloc_errors(self):
        n = self.store.numel
        world = self.dp_world
        self._pad = padded_size(n, world)
        dev = self.device
        self._mbuf = torch.zeros(self._pad, dtype=torch.float32, device=dev)
        self._werr = torch.zeros(self._pad, dtype=torch.float32, device=dev)
        self._serr = torch.zeros(self._pad // world, dtype=torch.float32, device=dev)

    @torch.no_grad()
    def step(self, closure=None):
        self.n_steps += 1
        ob = self.ob
        if not self.compressing:
            if self.ob_kind == "onebit_lamb":
                ok = self._lamb_warmup_step()
            else:
                ok = super().step()
            if self.n_steps >= getattr(ob, "freeze_step", 1 << 62):
                self.compressing = True
                if self.ob_kind == "onebit_lamb":
                    self.lamb_coeff = dict(self.lamb_last)
            return ok
        return self._compressed_step()

    def _lamb_warmup_step(self):
        s = self.store
        g0 = self.param_groups[0]
        b1, b2 = g0.get("betas", (0.9, 0.999))
        eps, wd, lr = g0.get("eps", 1e-8), g0.get("weight_decay", 0.0), g0["lr"]
        inv = 1.0 / (self.dp_world * self.loss_scaler.loss_scale)
        if "exp_avg" not in s.states:
            s.states["exp_avg"] = torch.zeros_like(s.master)
            s.states["exp_avg_sq"] = torch.zeros_like(s.master)
        m_all, v_all = s.states["exp_avg"], s.states["exp_avg_sq"]
        g_all = s.grad.float() * inv
        m_all.mul_(b1).add_(g_all, alpha=1 - b1)
        v_all.mul_(b2).addcmul_(g_all, g_all, value=1 - b2)
        for (p, w), (_, m), (_, v) in zip(self._param_views(s.master), self._param_views(m_all),
                                          self._param_views(v_all)):
            upd = m / (v.sqrt() + eps)
            if wd:
                upd = upd + wd * w
            wn, un = w.norm(), upd.norm()
            coeff = (wn / un).clamp(self.ob.min_coeff, self.ob.max_coeff) if wn > 0 and un > 0 else \
                torch.ones((), device=w.device)
            self.lamb_last[id(p)] = float(coeff)
            w.add_(upd, alpha=-lr * float(coeff))
        s.lp.copy_(s.master)
        self._post_step_gather()
        self.zero_grad()
        return True

    def _compressed_step(self):
        s = self.store
        ob = self.ob
        g0 = self.param_groups[0]
        b1, b2 = g0.get("betas", (0.9, 0.999))
        eps, wd, lr = g0.get("eps", 1e-8), g0.get("weight_decay", 0.0), g0["lr"]
        if self._werr is None:
            self._alloc_errors()
        if "exp_avg" not in s.states:
            s.states["exp_avg"] = torch.zeros_like(s.master)
            s.states["exp_avg_sq"] = torch.zeros_like(s.master)
        m, v = s.states["exp_avg"], s.states["exp_avg_sq"]
        g = s.grad.float() * (1.0 / self.loss_scaler.loss_scale)  # LOCAL gradient (no all-reduce)
        n = s.numel
        buf = self._mbuf
        if self.ob_kind == "zero_one_adam" and not self.var_frozen:
            # 0/1 Adam before the variance freezes: on variance steps (a doubling interval) the gradient is
            # all-reduced exactly and updates m and v; on the others the gradient itself is 1-bit all-reduced
            if self.n_steps % self.var_interval == 0:
                from ... import comm as dist
                dist.all_reduce(g, group=self.dp_group)
                g.div_(self.dp_world)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                m.mul_(b1).add_(g, alpha=1 - b1)
                self.var_counter += 1
                if self.var_counter == ob.var_update_scaler:
                    self.var_counter = 0
                    self.var_interval *= 2
            else:
                buf[:n].copy_(g)
                buf[n:].zero_()
                compressed_allreduce(buf, self._werr, self._serr, self.dp_group)
                m.mul_(b1).add_(buf[:n], alpha=1 - b1)
            if self.n_steps >= ob.var_freeze_step:
                self.var_frozen = True
        else:
            # frozen variance: local momentum, ONE compressed all-reduce of the momentum
            m.mul_(b1).add_(g, alpha=1 - b1)
            buf[:n].copy_(m)
            buf[n:].zero_()
            compressed_allreduce(buf, self._werr, self._serr, self.dp_group)
            m.copy_(buf[:n])
        seen = v > 0  # automatic exp_avg_mask: coordinates that never had a gradient are not moved
        if self.ob_kind == "onebit_lamb":
            for (p, w), (_, mv), (_, vv) in zip(self._param_views(s.master), self._param_views(m),
                                                self._param_views(v)):
                upd = torch.where(vv > 0, mv / (vv.sqrt() + eps), torch.zeros_like(mv))
                if wd:
                    upd = upd + wd * w
                w.add_(upd, alpha=-lr * self.lamb_coeff.get(id(p), 1.0))
        else:
            upd = torch.where(seen, m / (v.sqrt() + eps), torch.zeros_like(m))
            if wd:
                upd.add_(s.master, alpha=wd)
            s.master.add_(upd, alpha=-lr)
        s.lp.copy_(s.master)
        self._post_step_gather()
        self.zero_grad()
        return True
