"""Move optimizer-owned device memory to pinned host memory between steps and back.

Reference parity: runtime/zero/offload_states.py (``OffloadStateTypeEnum`` :19, ``offload_adam_states`` :38)
and stage3.py ``offload_states``/``reload_states`` (:2848-2991), engine.py :3943/:3977. Typical use: free
HBM for a generation phase (RLHF) or another model, then ``reload_states()`` before the next step.
With the flat-shard store every state is ONE contiguous buffer, so each offload/reload is a single
pinned-memory DMA per state on a side stream.
"""
from enum import Enum

import torch

from .flat import AVAILABLE


class OffloadStateTypeEnum(str, Enum):
    optim_states = "optim_states"
    hp_params = "hp_params"
    lp_params = "lp_params"
    lp_grads = "lp_grads"
    contiguous_grad_buffer = "contiguous_grad_buffer"


ALL = tuple(OffloadStateTypeEnum)


def _to_host(t, pin, non_blocking):
    h = torch.empty(t.shape, dtype=t.dtype, device="cpu", pin_memory=pin and torch.cuda.is_available())
    h.copy_(t, non_blocking=non_blocking)
    return h


def offload_states(zopt, include=None, device="cpu", pin_memory=True, non_blocking=False):
    assert device == "cpu", "only host offload is supported"
    if getattr(zopt, "kind", None) == "generic":
        raise NotImplementedError("offload_states needs a fused optimizer (Adam/Lion/Adagrad) over the flat store")
    include = [OffloadStateTypeEnum(i) for i in (include or ALL)]
    s = zopt.store
    saved = getattr(zopt, "_offloaded_states", {})
    dev = s.lp.device
    empty = lambda dt: torch.empty(0, dtype=dt, device=dev)  # noqa: E731
    if OffloadStateTypeEnum.optim_states in include and s.states:
        saved["states"] = {k: _to_host(v, pin_memory, non_blocking) for k, v in s.states.items()}
        s.states = {k: empty(v.dtype) for k, v in s.states.items()}
    if OffloadStateTypeEnum.hp_params in include and s.master is not None and s.master.numel():
        saved["master"] = _to_host(s.master, pin_memory, non_blocking)
        s.master = empty(s.master.dtype)
    if (OffloadStateTypeEnum.lp_grads in include or OffloadStateTypeEnum.contiguous_grad_buffer in include) \
            and s.grad.numel():
        saved["grad"] = _to_host(s.grad, pin_memory, non_blocking)
        for u in zopt.units:
            u.unbind_grads()
            if u.direct or u.grad_full is not None:
                u.grad_full = None
        s.grad = empty(s.grad.dtype)
    if OffloadStateTypeEnum.lp_params in include and s.lp.numel():
        saved["lp"] = _to_host(s.lp, pin_memory, non_blocking)
        for u in zopt.units:
            if u.world == 1 or u.persistent:
                u.unbind_params(empty(s.lp.dtype))
                u.full = None
            u.shard_tensor = None
        s.lp = empty(s.lp.dtype)
    if non_blocking and torch.cuda.is_available():
        torch.cuda.current_stream().synchronize()
    zopt._offloaded_states = saved
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def reload_states(zopt, non_blocking=False):
    saved = getattr(zopt, "_offloaded_states", None)
    if not saved:
        return
    s = zopt.store
    dev = zopt.device
    if "states" in saved:
        s.states = {k: v.to(dev, non_blocking=non_blocking) for k, v in saved["states"].items()}
    if "master" in saved:
        s.master = saved["master"].to(dev, non_blocking=non_blocking)
    if "lp" in saved:
        s.lp = saved["lp"].to(dev, non_blocking=non_blocking)
        for u in zopt.units:
            lp = s.lp_slice(u)
            u.shard_tensor = lp
            for p in u.params:
                p.ds_tensor = lp
            if u.world == 1:
                u.full = lp
                u.bind_params(lp)
                u.status = AVAILABLE
            elif u.persistent:
                full = torch.empty(u.padded, dtype=s.lp.dtype, device=dev)
                u.full = full
                u.bind_params(full)
                u.status = AVAILABLE
        zopt._post_step_gather()
    if "grad" in saved:
        s.grad = saved["grad"].to(dev, non_blocking=non_blocking)
        for u in zopt.units:
            if u.direct:
                u.grad_full = s.grad_slice(u)
                u.bind_grads(u.grad_full)
            elif u.persistent or u.world == 1:
                u.grad_full = torch.zeros(u.padded, dtype=zopt.dtype, device=dev)
                u.bind_grads(u.grad_full)
    if non_blocking and torch.cuda.is_available():
        torch.cuda.current_stream().synchronize()
    zopt._offloaded_states = {}
