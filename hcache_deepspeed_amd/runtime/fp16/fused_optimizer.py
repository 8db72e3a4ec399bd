"""Standalone mixed-precision optimizer wrappers (no ZeRO): fp16 with loss scaling, bf16 with fp32 master.

Reference parity: runtime/fp16/fused_optimizer.py (``FP16_Optimizer`` :33 -- flat fp32 master per param group,
dynamic/static loss scaling, overflow skip, grad clipping), runtime/fp16/unfused_optimizer.py
(``FP16_UnfusedOptimizer`` :24 -- per-parameter fp32 masters, used for LAMB) and runtime/bf16_optimizer.py
(``BF16_Optimizer`` :35 -- bf16 params, fp32 grad accumulation and master). Inside the engine every stage
(including 0) runs through the flat-shard ZeroOptimizer (runtime/zero/optimizer.py) which already implements all
of this on one contiguous store; these classes give user code the reference's standalone wrapper API over any
torch optimizer (FusedAdam's HIP multi-tensor kernel when passed one).
"""
import torch
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from ..utils import clip_grad_norm_
from .loss_scaler import CreateLossScaler


class _MasterWeightOptimizer:
    """Shared machinery: lp params <-> fp32 masters, overflow check, clipping, state dict."""

    flat = True

    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False, initial_dynamic_scale=2**32,
                 dynamic_loss_args=None, clip_grad=0.0, mpu=None, lp_dtype=torch.float16, use_scaler=True):
        self.optimizer = init_optimizer
        self.clip_grad = clip_grad
        self.mpu = mpu
        self.lp_groups, self.fp32_groups = [], []
        for g in self.optimizer.param_groups:
            lp = [p for p in g["params"] if p.requires_grad]
            self.lp_groups.append(lp)
            if self.flat:
                master = _flatten_dense_tensors([p.detach().float() for p in lp]).clone().requires_grad_(True)
                g["params"] = [master]
                self.fp32_groups.append([master])
            else:
                masters = [p.detach().float().clone().requires_grad_(True) for p in lp]
                g["params"] = masters
                self.fp32_groups.append(masters)
        # re-key optimizer state onto the masters
        self.optimizer.state = type(self.optimizer.state)()
        dyn_args = dict(dynamic_loss_args or {})
        if dynamic_loss_scale:
            dyn_args.setdefault("init_scale", initial_dynamic_scale)
        self.loss_scaler = CreateLossScaler(torch.float16 if use_scaler else torch.bfloat16, static_loss_scale,
                                            dynamic_loss_scale, dyn_args) if use_scaler else None
        self.overflow = False

    # -- reference API -----------------------------------------------------------------------
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    @property
    def cur_scale(self):
        return self.loss_scaler.cur_scale if self.loss_scaler is not None else 1.0

    @property
    def loss_scale(self):
        return self.cur_scale

    def zero_grad(self, set_to_none=True):
        for group in self.lp_groups:
            for p in group:
                if set_to_none:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.detach_().zero_()

    def backward(self, loss, create_graph=False, retain_graph=False):
        (loss.float() * self.cur_scale).backward(create_graph=create_graph, retain_graph=retain_graph)

    def _lp_grads_to_master(self):
        overflow = False
        for lp, masters in zip(self.lp_groups, self.fp32_groups):
            grads = [(p.grad if p.grad is not None else torch.zeros_like(p)).float() for p in lp]
            if self.flat:
                g = _flatten_dense_tensors(grads)
                masters[0].grad = g
                overflow |= not bool(torch.isfinite(g).all())
            else:
                for m, g in zip(masters, grads):
                    m.grad = g
                    overflow |= not bool(torch.isfinite(g).all())
        return overflow

    def _master_to_lp(self):
        with torch.no_grad():
            for lp, masters in zip(self.lp_groups, self.fp32_groups):
                vals = _unflatten_dense_tensors(masters[0].data, lp) if self.flat else [m.data for m in masters]
                for p, v in zip(lp, vals):
                    p.data.copy_(v)

    def step(self, closure=None):
        self.overflow = self._lp_grads_to_master()
        if self.loss_scaler is not None:
            self.loss_scaler.update_scale(self.overflow)
        if self.overflow:
            for masters in self.fp32_groups:
                for m in masters:
                    m.grad = None
            return False
        inv = 1.0 / self.cur_scale if self.loss_scaler is not None else 1.0
        masters = [m for ms in self.fp32_groups for m in ms]
        if inv != 1.0:
            for m in masters:
                m.grad.mul_(inv)
        if self.clip_grad > 0:
            clip_grad_norm_(masters, self.clip_grad, mpu=self.mpu)
        self.optimizer.step()
        for m in masters:
            m.grad = None
        self._master_to_lp()
        return True

    def refresh_fp32_params(self):
        with torch.no_grad():
            for lp, masters in zip(self.lp_groups, self.fp32_groups):
                if self.flat:
                    masters[0].data.copy_(_flatten_dense_tensors([p.detach().float() for p in lp]))
                else:
                    for m, p in zip(masters, lp):
                        m.data.copy_(p.data.float())

    def state_dict(self):
        sd = {"optimizer_state_dict": self.optimizer.state_dict(), "fp32_groups": [[m.detach().clone() for m in ms]
                                                                                 for ms in self.fp32_groups],
              "clip_grad": self.clip_grad, "overflow": self.overflow}
        if self.loss_scaler is not None:
            sd["loss_scaler"] = self.loss_scaler.state_dict()
        return sd

    def load_state_dict(self, state_dict, load_optimizer_states=True):
        if load_optimizer_states:
            self.optimizer.load_state_dict(state_dict["optimizer_state_dict"])
        if self.loss_scaler is not None and "loss_scaler" in state_dict:
            self.loss_scaler.load_state_dict(state_dict["loss_scaler"])
        self.clip_grad = state_dict.get("clip_grad", self.clip_grad)
        with torch.no_grad():
            for ms, saved in zip(self.fp32_groups, state_dict["fp32_groups"]):
                for m, s in zip(ms, saved):
                    m.data.copy_(s)
        self._master_to_lp()


class FP16_Optimizer(_MasterWeightOptimizer):
    """fp16 params, flat fp32 master per group, static or dynamic loss scaling (reference :33)."""

    def __init__(self, init_optimizer, deepspeed=None, static_loss_scale=1.0, dynamic_loss_scale=False,
                 initial_dynamic_scale=2**32, dynamic_loss_args=None, verbose=True, mpu=None, clip_grad=0.0,
                 fused_adam_legacy=False, has_moe_layers=False, timers=None):
        super().__init__(init_optimizer, static_loss_scale, dynamic_loss_scale, initial_dynamic_scale,
                         dynamic_loss_args, clip_grad, mpu, torch.float16, use_scaler=True)


class FP16_UnfusedOptimizer(FP16_Optimizer):
    """Per-parameter fp32 masters (reference unfused_optimizer.py:24; needed by LAMB's per-tensor trust ratio)."""
    flat = False


class BF16_Optimizer(_MasterWeightOptimizer):
    """bf16 params, fp32 grads and master, no loss scaling (reference bf16_optimizer.py:35)."""

    def __init__(self, init_optimizer, param_names=None, mpu=None, clip_grad=0.0, norm_type=2,
                 allgather_bucket_size=5000000000, dp_process_group=None, timers=None, grad_acc_dtype=None,
                 graph_harvesting=False, immediate_grad_update=False, has_moe_layers=False):
        super().__init__(init_optimizer, clip_grad=clip_grad, mpu=mpu, lp_dtype=torch.bfloat16, use_scaler=False)
