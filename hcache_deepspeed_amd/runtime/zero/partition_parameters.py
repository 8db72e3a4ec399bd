"""``zero.Init`` / ``GatheredParameters`` for the flat-shard ZeRO-3 (reference: runtime/zero/partition_parameters.py,
``Init`` :302-615 patching module construction, ``GatheredParameters`` :2120-2256).

``Init`` constructs the model on the ``meta`` device (no memory anywhere); the ZeRO-3 optimizer then
materialises ONE unit at a time on the GPU (``materialize_unit``), runs the module's initialiser with a
per-unit seed identical on every rank, keeps its own shard and frees the rest. A 70B model therefore
never exists in full on any device or host. ``GatheredParameters`` temporarily gathers the units that own
the given parameters (e.g. to read or re-initialise weights) and writes modifications back to every
rank's shard on exit.
"""
import contextlib

import torch
import torch.nn as nn

from ... import comm as dist


class Init(contextlib.ContextDecorator):
    """Construct modules on the meta device; ZeRO-3 materialises them shard by shard."""

    _active = 0

    def __init__(self, module=None, data_parallel_group=None, mem_efficient_linear=True, remote_device=None,
                 pin_memory=False, config_dict_or_path=None, config=None, enabled=True, dtype=None, mpu=None,
                 zero_param_parallel_group=None, zero_quantized_weights=False, zero_quantized_nontrainable_weights=False,
                 sequence_data_parallel_group=None, param_swapper=None):
        self.enabled = enabled
        self.dtype = dtype
        self._ctx = None
        if module is not None and enabled:
            # already-constructed module: nothing to do, sharding happens in deepspeed.initialize
            pass

    def __enter__(self):
        if not self.enabled:
            return self
        Init._active += 1
        self._ctx = torch.device("meta")
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        self._ctx.__exit__(*exc)
        Init._active -= 1
        return False


def is_zero_init_active():
    return Init._active > 0


def materialize_unit(unit, device, dtype, seed):
    """Give meta parameters of one unit real storage and initialise them deterministically.

    Returns {id(old_meta_param): new_param}; meta tensors cannot be re-pointed in place, so the new
    Parameter objects replace the old ones in their modules and the caller swaps its references.
    """
    metas = [p for p in unit.params if p.is_meta]
    if not metas:
        return {}
    repl = {}
    mods = []
    mine = {id(p) for p in metas}
    for m in unit.module.modules():
        touched = False
        for n, p in list(m._parameters.items()):
            if p is not None and p.is_meta and id(p) in mine:
                if id(p) not in repl:
                    new = nn.Parameter(torch.empty(p.shape, dtype=dtype or p.dtype, device=device),
                                       requires_grad=p.requires_grad)
                    new.__dict__.update(p.__dict__)  # tags: allreduce/group_name/tensor-parallel flags
                    repl[id(p)] = new
                m._parameters[n] = repl[id(p)]
                touched = True
        for n, b in list(m._buffers.items()):
            if b is not None and b.is_meta:
                m._buffers[n] = torch.zeros(b.shape, dtype=b.dtype, device=device)
        if touched:
            mods.append(m)
    with torch.random.fork_rng(devices=[device] if device.type == "cuda" else []):
        torch.manual_seed(seed)
        if device.type == "cuda":
            torch.cuda.manual_seed(seed)
        with torch.no_grad():
            for m in mods:
                if hasattr(m, "reset_parameters"):
                    m.reset_parameters()
                elif hasattr(m, "_init_weights"):
                    m._init_weights(m)
                else:
                    for p in m.parameters(recurse=False):
                        nn.init.normal_(p, std=0.02)
    return repl


def _zero_of(p):
    return getattr(p, "_hds_zero", None)


class GatheredParameters:
    """Gather the full values of ZeRO-3 partitioned parameters inside the context.

    ``modifier_rank``: rank whose in-context modifications are broadcast and written back to all shards.
    """

    def __init__(self, params, modifier_rank=None, fwd_module=None, enabled=True):
        if isinstance(params, nn.Parameter) or isinstance(params, torch.Tensor):
            params = [params]
        self.params = list(params) if params is not None else []
        self.modifier_rank = modifier_rank
        self.enabled = enabled
        self.units = []

    def __enter__(self):
        if not self.enabled:
            return self
        seen = set()
        for p in self.params:
            z = _zero_of(p)
            if z is None:
                continue
            u, _ = z.param_to_unit[id(p)]
            if id(u) not in seen:
                seen.add(id(u))
                self.units.append((z, u))
        for z, u in self.units:
            z._gather(u, wait=True)
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        with torch.no_grad():
            for z, u in self.units:
                if self.modifier_rank is not None:
                    if u.world > 1:
                        src = dist.get_global_rank(u.dp_group, self.modifier_rank) if u.dp_group is not None \
                            else self.modifier_rank
                        dist.broadcast(u.full, src, group=u.dp_group)
                    lp = z.store.lp_slice(u)
                    if u.full.data_ptr() != lp.data_ptr():
                        lp.copy_(u.full[u.rank * u.shard:(u.rank + 1) * u.shard])
                    z.store.master[u.store_off:u.store_off + u.shard].copy_(lp)
                if not u.persistent and z._partitioned(u) and not z.in_backward:
                    z._release(u)
        self.units = []
        return False


def register_external_parameter(module, parameter):
    """Compatibility no-op: units used outside their module are kept in the persistent root unit."""
    if not hasattr(module, "_external_params"):
        module._external_params = {}
    module._external_params[id(parameter)] = parameter


def unregister_external_parameter(module, parameter):
    if hasattr(module, "_external_params"):
        module._external_params.pop(id(parameter), None)


def set_z3_leaf_modules(model, leaf_module_classes):
    """Treat every instance of the given classes as ONE ZeRO-3 fetch unit (reference utils/z3_leaf_module.py)."""
    cur = tuple(getattr(model, "_z3_leaf_modules", ()))
    model._z3_leaf_modules = cur + tuple(leaf_module_classes)
    return [m for m in model.modules() if isinstance(m, tuple(leaf_module_classes))]


def get_z3_leaf_modules(model):
    return [m for m in model.modules() if isinstance(m, tuple(getattr(model, "_z3_leaf_modules", ())))]
