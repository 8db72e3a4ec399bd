"""Full / local views of a parameter's high-precision state held in the flat ZeRO store.

Reference parity: utils/tensor_fragment.py (``safe_get_full_fp32_param`` :132, ``safe_set_full_fp32_param``,
``safe_get_full_optimizer_state`` :164, ``safe_set_full_optimizer_state``, ``safe_get_full_grad`` :199,
``safe_set_full_grad``, ``safe_get_local_*`` / ``safe_set_local_*`` :243-310). Each parameter is a
contiguous range of its unit's rank-major flat buffer; the "local" fragment is the intersection of that
range with this rank's shard, the "full" value is ONE all-gather of the unit's shard (collective over the
unit's data-parallel group: call on every rank).
"""
from dataclasses import dataclass

import torch

from .. import comm as dist


@dataclass
class fragment_address:
    """Where one parameter's fragment sits inside a rank's flat optimizer partition (reference
    utils/tensor_fragment.py:13). Written into ZeRO-1/2 ``param_slice_mappings``."""
    numel: int
    start: int


torch.serialization.add_safe_globals([fragment_address])

_GRAD = "__grad__"
_FP32 = "__fp32__"


def _zopt(param):
    return getattr(param, "_hds_zero", None)


def _buffer(z, key):
    if key != _GRAD and getattr(z, "state_offload", None) is not None:
        z.state_offload.wait()
    s = z.store
    if key == _FP32:
        return s.master
    if key == _GRAD:
        return s.grad
    return s.states.get(key)


def _local_range(z, u, i):
    """(param-relative [a, b), store [lo, hi)) of this rank's fragment of param i of unit u."""
    lo_sh, hi_sh = u.rank * u.shard, (u.rank + 1) * u.shard
    p0, p1 = u.offsets[i], u.offsets[i] + u.numels[i]
    a, b = max(lo_sh, p0), min(hi_sh, p1)
    if a >= b:
        return None
    return (a - p0, b - p0), (u.store_off + a - lo_sh, u.store_off + b - lo_sh)


def _full_unit(z, u, key):
    buf = _buffer(z, key)
    if buf is None:
        return None
    mine = buf[u.store_off:u.store_off + u.shard]
    if u.world == 1:
        return mine
    full = torch.empty(u.padded, dtype=mine.dtype, device=mine.device)
    dist.all_gather_into_tensor(full, mine.contiguous(), group=u.dp_group)
    return full


def _get_full(param, key):
    z = _zopt(param)
    if z is None:
        if key == _GRAD:
            return None if param.grad is None else param.grad.float()
        return param.detach().float() if key == _FP32 else None
    u, i = z.param_to_unit[id(param)]
    full = _full_unit(z, u, key)
    if full is None:
        return None
    out = u.param_view(full, i).clone().float()
    if key == _GRAD:
        out.mul_(1.0 / (z.layout_world_for_avg() * z.loss_scaler.loss_scale))
    return out


def _set_full(param, value, key):
    z = _zopt(param)
    if z is None:
        if key == _FP32:
            param.data.copy_(value)
        elif key == _GRAD:
            param.grad = value.to(param.dtype).clone()
        return
    u, i = z.param_to_unit[id(param)]
    r = _local_range(z, u, i)
    if r is not None:
        (a, b), (lo, hi) = r
        buf = _buffer(z, key)
        src = value.reshape(-1)[a:b].to(buf.dtype)
        if key == _GRAD:
            src = src * (z.layout_world_for_avg() * z.loss_scaler.loss_scale)
        buf[lo:hi].copy_(src)
        if key == _FP32:
            z._lp_wait()
            z.store.lp[lo:hi].copy_(buf[lo:hi])
            z._lp_written(u)
    if key == _FP32:
        z._post_step_gather()  # collective: every rank refreshes the gathered copies


def safe_get_full_fp32_param(param):
    return _get_full(param, _FP32)


def safe_set_full_fp32_param(param, value):
    _set_full(param, value, _FP32)


def safe_get_full_optimizer_state(param, optim_state_key):
    return _get_full(param, optim_state_key)


def safe_set_full_optimizer_state(param, value, optim_state_key):
    _set_full(param, value, optim_state_key)


def safe_get_full_grad(param):
    """Averaged (over data parallel) fp32 gradient; valid between backward and step."""
    return _get_full(param, _GRAD)


def safe_set_full_grad(param, value):
    _set_full(param, value, _GRAD)


def _get_local(param, key):
    z = _zopt(param)
    if z is None:
        return _get_full(param, key)
    u, i = z.param_to_unit[id(param)]
    r = _local_range(z, u, i)
    if r is None:
        return None
    _, (lo, hi) = r
    buf = _buffer(z, key)
    return None if buf is None else buf[lo:hi].float().clone()


def _set_local(param, value, key):
    z = _zopt(param)
    if z is None:
        return _set_full(param, value, key)
    u, i = z.param_to_unit[id(param)]
    r = _local_range(z, u, i)
    if r is None:
        return
    _, (lo, hi) = r
    buf = _buffer(z, key)
    buf[lo:hi].copy_(value.reshape(-1).to(buf.dtype))
    if key == _FP32:
        z._lp_wait()
        z.store.lp[lo:hi].copy_(buf[lo:hi])
        z._lp_written(u)


def safe_get_local_grad(param):
    return _get_local(param, _GRAD)


def safe_set_local_grad(param, value):
    _set_local(param, value, _GRAD)


def safe_get_local_fp32_param(param):
    return _get_local(param, _FP32)


def safe_set_local_fp32_param(param, value):
    _set_local(param, value, _FP32)


def safe_get_local_optimizer_state(param, optim_state_key):
    return _get_local(param, optim_state_key)


def safe_set_local_optimizer_state(param, value, optim_state_key):
    _set_local(param, value, optim_state_key)


# ---------------------------------------------------------------------------------------------------------------------
# hp-param helpers under the reference's names (utils/tensor_fragment.py get_full_hp_param / set_full_hp_param /
# get_full_hp_grad / set_full_hp_grad / get_hp_fragment_mapping / map_to_flat_opt_states, mixed_precision_linkage.py
# link_hp_params / lazy_init_hp_params_optimizer_state). The reference links every low-precision parameter to its
# fragment of a flat fp32 partition and binds these as methods; here the parameter already knows its unit and offset
# in the flat store, so the functions take the parameter and ``link_hp_params`` binds them the same way.
# ---------------------------------------------------------------------------------------------------------------------
def get_full_hp_param(param, optim_state_key=None):
    """The full fp32 value of ``param`` (or of its optimizer state ``optim_state_key``). Collective."""
    return _get_full(param, _FP32 if optim_state_key is None else optim_state_key)


def set_full_hp_param(param, value, optim_state_key=None):
    """Write the full fp32 value (or optimizer state) of ``param``; each rank keeps its fragment. Collective."""
    _set_full(param, value, _FP32 if optim_state_key is None else optim_state_key)


def get_full_hp_grad(param):
    return _get_full(param, _GRAD)


def set_full_hp_grad(param, value):
    _set_full(param, value, _GRAD)


def get_hp_fragment_mapping(param):
    """{"lp_fragment_address", "hp_fragment_address"}: where this rank's fragment of ``param`` sits inside the
    parameter (lp) and inside this rank's flat fp32 partition (hp); None when this rank holds none of it."""
    z = _zopt(param)
    if z is None:
        return None
    u, i = z.param_to_unit[id(param)]
    r = _local_range(z, u, i)
    if r is None:
        return None
    (a, b), (lo, hi) = r
    return {"lp_fragment_address": fragment_address(numel=b - a, start=a),
            "hp_fragment_address": fragment_address(numel=hi - lo, start=lo)}


def map_to_flat_opt_states(flat_hp_tensor, lp_tensors, optim_state, opt_keys):
    """Concatenate the per-parameter optimizer states of ``lp_tensors`` into flat states keyed by
    ``flat_hp_tensor`` (a torch optimizer's per-parameter state -> the flat layout the ZeRO store uses)."""
    merged = optim_state.setdefault(flat_hp_tensor, {})
    for key in opt_keys:
        parts = [optim_state[lp][key].reshape(-1) for lp in lp_tensors if lp in optim_state and key in optim_state[lp]]
        if parts:
            merged[key] = torch.cat(parts)
    return merged


def link_hp_params(lp_param_list, *args, **kwargs):
    """Bind ``get_full_hp_param`` / ``set_full_hp_param`` / ``get_full_hp_grad`` / ``set_full_hp_grad`` /
    ``get_hp_fragment_mapping`` as methods of every parameter (the reference's linkage; the extra arguments of its
    signature -- flat partition, gradient dicts, partition bounds -- are implied by the flat store here)."""
    import functools
    for p in lp_param_list:
        p.get_full_hp_param = functools.partial(get_full_hp_param, p)
        p.set_full_hp_param = functools.partial(set_full_hp_param, p)
        p.get_full_hp_grad = functools.partial(get_full_hp_grad, p)
        p.set_full_hp_grad = functools.partial(set_full_hp_grad, p)
        p.get_hp_fragment_mapping = functools.partial(get_hp_fragment_mapping, p)
    return lp_param_list


def lazy_init_hp_params_optimizer_state(lp_param_list, *args, **kwargs):
    """The reference creates the optimizer-state fragments of linked parameters after the first step; the flat store
    creates its states with the optimizer, so this only makes sure they are resident (state offload) for readers."""
    seen = set()
    for p in lp_param_list:
        z = _zopt(p)
        if z is not None and id(z) not in seen:
            seen.add(id(z))
            so = getattr(z, "state_offload", None)
            if so is not None:
                so.wait()
