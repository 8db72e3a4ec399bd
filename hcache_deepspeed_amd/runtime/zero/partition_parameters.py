"""``zero.Init`` / ``GatheredParameters`` for the flat-shard ZeRO-3 (reference: runtime/zero/partition_parameters.py,
``Init`` :302-615 / :1108-1472 partitioning every parameter as its module finishes ``__init__``,
``GatheredParameters`` :2120-2256).

``Init`` semantics (same contract as the reference):

* every module constructed inside the context is built normally (on the local GPU by default, so its own
  initialiser runs at full speed); its parameters are then broadcast from data-parallel rank 0 and cut into
  ``ceil(numel / world)``-element partitions; the rank keeps its partition on ``remote_device`` (``"cpu"`` /
  ``"nvme"``: host memory, pinned with ``pin_memory``) and the parameter's storage is freed
  (``p.numel() == 0``, ``p.ds_shape`` / ``p.ds_numel`` keep the logical size).
* WHEN: at the end of the outermost constructor (so a parent's ``__init__`` may still write its children's
  weights), unless the not-yet-partitioned parameters exceed ``defer_bytes`` (default: a quarter of the free
  device memory): then every module that has finished its own ``__init__`` is partitioned right away, which
  bounds peak memory for 70B-class models the way the reference's per-module partitioning does.
* values set inside ``__init__`` survive; weights loaded inside the context -- ``model.load_state_dict(sd)``
  (a load pre-hook writes each rank's slice) or ``GatheredParameters(..., modifier_rank=0)`` -- survive too.
* ``deepspeed.initialize`` then moves the per-parameter partitions into the flat-unit layout of the ZeRO-3
  optimizer with one reduce-scatter per unit (the slices are disjoint, so the sum is exact); ZeRO-0/1/2
  gather the parameters back instead.
"""
import contextlib
import math

import torch
import torch.nn as nn

from ... import comm as dist


def _all_subclasses(cls):
    out, todo = set(), [cls]
    while todo:
        c = todo.pop()
        for s in c.__subclasses__():
            if s not in out:
                out.add(s)
                todo.append(s)
    return out


def is_init_partitioned(p):
    return getattr(p, "_hds_part", None) is not None


class Init(contextlib.ContextDecorator):
    """Partition parameters at module construction (see module docstring)."""

    _active = 0
    _current = None

    def __init__(self, module=None, data_parallel_group=None, mem_efficient_linear=True, remote_device=None,
                 pin_memory=False, config_dict_or_path=None, config=None, enabled=True, dtype=None, mpu=None,
                 zero_param_parallel_group=None, zero_quantized_weights=False, zero_quantized_nontrainable_weights=False,
                 sequence_data_parallel_group=None, param_swapper=None, defer_bytes=None):
        self.enabled = enabled
        self.defer_bytes = defer_bytes
        self._depth = 0
        self._pending = []
        self._pending_bytes = 0
        self.dtype = dtype
        self.group = data_parallel_group or sequence_data_parallel_group
        self.remote = remote_device if remote_device in ("cpu", "nvme") else None
        self.pin = bool(pin_memory)
        self._patched = []
        self._dev_ctx = None
        if module is not None and enabled:
            # an already-built module: partition it now (reference Init(module=...))
            dist.init_distributed(verbose=False)
            for m in module.modules():
                self._partition_module(m)

    # ---- context --------------------------------------------------------------------------
    def __enter__(self):
        if not self.enabled:
            return self
        dist.init_distributed(verbose=False)
        Init._active += 1
        self._prev, Init._current = Init._current, self
        if torch.cuda.is_available():
            self._dev_ctx = torch.device("cuda", torch.cuda.current_device())
            self._dev_ctx.__enter__()
            if self.defer_bytes is None:
                self.defer_bytes = torch.cuda.mem_get_info()[0] // 4
        elif self.defer_bytes is None:
            self.defer_bytes = 8 << 30
        self._patch()
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        self._flush()
        self._unpatch()
        if self._dev_ctx is not None:
            self._dev_ctx.__exit__(*exc)
            self._dev_ctx = None
        Init._current = self._prev
        Init._active -= 1
        return False

    def _patch(self):
        """Wrap ``__init__`` of every nn.Module subclass (and of subclasses defined inside the context)."""
        ctx = self

        def wrap(cls):
            orig = cls.__dict__.get("__init__")
            if orig is None or getattr(orig, "_hds_wrapped", False):
                return

            def __init__(self, *a, **k):
                depth = self.__dict__.get("_hds_init_depth", 0)
                object.__setattr__(self, "_hds_init_depth", depth + 1)
                ctx._depth += 1
                try:
                    orig(self, *a, **k)
                finally:
                    object.__setattr__(self, "_hds_init_depth", depth)
                    ctx._depth -= 1
                if depth == 0:
                    ctx._module_done(self)

            __init__._hds_wrapped = True
            __init__.__wrapped__ = orig
            cls.__init__ = __init__
            ctx._patched.append((cls, orig))

        for c in [nn.Module] + sorted(_all_subclasses(nn.Module), key=lambda c: c.__qualname__):
            wrap(c)
        prev_isc = nn.Module.__dict__.get("__init_subclass__")

        @classmethod
        def __init_subclass__(cls, **kw):
            super(nn.Module, cls).__init_subclass__(**kw)
            wrap(cls)

        nn.Module.__init_subclass__ = __init_subclass__
        self._prev_isc = prev_isc

    def _unpatch(self):
        for cls, orig in reversed(self._patched):
            cls.__init__ = orig
        self._patched = []
        if self._prev_isc is None:
            try:
                del nn.Module.__init_subclass__
            except AttributeError:
                pass
        else:
            nn.Module.__init_subclass__ = self._prev_isc

    # ---- partitioning ---------------------------------------------------------------------
    def _world_rank(self):
        if not dist.is_initialized():
            return 1, 0
        return dist.get_world_size(self.group), dist.get_rank(self.group)

    def _module_done(self, m):
        self._pending.append(m)
        self._pending_bytes += sum(p.numel() * p.element_size() for p in m.parameters(recurse=False))
        if self._depth == 0 or self._pending_bytes > self.defer_bytes:
            self._flush()

    def _flush(self):
        pending, self._pending, self._pending_bytes = self._pending, [], 0
        for m in pending:
            self._partition_module(m)

    def _partition_module(self, m):
        params = [(n, p) for n, p in m.named_parameters(recurse=True) if not is_init_partitioned(p)]
        if not params:
            return
        for _, p in params:
            self._partition_param(p)
        if not getattr(m, "_hds_init_load_hook", False):
            m._register_load_state_dict_pre_hook(_load_into_partitions, with_module=True)
            m._hds_init_load_hook = True

    def _partition_param(self, p):
        W, r = self._world_rank()
        with torch.no_grad():
            data = p.data
            if W > 1:
                src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
                dist.broadcast(data, src, group=self.group)  # identical initial weights on every rank
            flat = data.reshape(-1)
            n = flat.numel()
            pn = math.ceil(n / W)
            dev = torch.device("cpu") if self.remote is not None else data.device
            part = torch.zeros(pn, dtype=self.dtype or data.dtype, device=dev,
                               pin_memory=self.pin and dev.type == "cpu" and torch.cuda.is_available())
            lo, hi = r * pn, min(n, (r + 1) * pn)
            if hi > lo:
                part[:hi - lo].copy_(flat[lo:hi])
        p.ds_shape = p.shape
        p.ds_numel = n
        p._hds_part = part
        p._hds_part_group = self.group
        p._hds_part_world = W
        p._hds_part_rank = r
        p.ds_status = 0
        p.data = torch.empty(0, dtype=data.dtype, device=data.device)


def is_zero_init_active():
    return Init._active > 0


def _load_into_partitions(module, state_dict, prefix, *args):
    """load_state_dict pre-hook of Init-partitioned modules: each rank writes its slice of every incoming full
    tensor into its partition; the entry is replaced by an empty tensor matching the (empty) parameter."""
    for name, p in module._parameters.items():
        key = prefix + name
        if p is None or key not in state_dict or not is_init_partitioned(p):
            continue
        t = state_dict[key]
        if tuple(t.shape) != tuple(p.ds_shape):
            continue  # let torch report the shape mismatch
        flat = t.reshape(-1)
        part = p._hds_part
        pn = part.numel()
        lo, hi = p._hds_part_rank * pn, min(flat.numel(), (p._hds_part_rank + 1) * pn)
        with torch.no_grad():
            part.zero_()
            if hi > lo:
                part[:hi - lo].copy_(flat[lo:hi])
        state_dict[key] = torch.empty(0, dtype=p.dtype, device=p.device)


def gather_init_param(p):
    """Full value of an Init-partitioned parameter (all-gather of the per-rank partitions)."""
    part = p._hds_part
    W = p._hds_part_world
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    src = part.to(dev)
    if W > 1:
        full = torch.empty(W * part.numel(), dtype=part.dtype, device=dev)
        dist.all_gather_into_tensor(full, src, group=p._hds_part_group)
    else:
        full = src
    return full[:p.ds_numel].view(p.ds_shape)


def unpartition_init_param(p, dtype=None, device=None):
    """Turn an Init-partitioned parameter back into a normal full parameter (ZeRO-0/1/2 engines)."""
    full = gather_init_param(p)
    p.data = full.to(dtype=dtype or full.dtype, device=device or full.device).clone()
    for a in ("_hds_part", "_hds_part_group", "_hds_part_world", "_hds_part_rank"):
        p.__dict__.pop(a, None)


def _zero_of(p):
    return getattr(p, "_hds_zero", None)


class GatheredParameters:
    """Gather the full values of ZeRO-3 partitioned parameters inside the context.

    Works both before ``deepspeed.initialize`` (parameters partitioned by ``zero.Init``) and after it (flat
    ZeRO-3 units). ``modifier_rank``: rank whose in-context modifications are broadcast and written back to every
    rank's partition.
    """

    def __init__(self, params, modifier_rank=None, fwd_module=None, enabled=True):
        if isinstance(params, nn.Parameter) or isinstance(params, torch.Tensor):
            params = [params]
        self.params = list(params) if params is not None else []
        self.modifier_rank = modifier_rank
        self.enabled = enabled
        self.units = []
        self.init_params = []

    def __enter__(self):
        if not self.enabled:
            return self
        seen = set()
        for p in self.params:
            z = _zero_of(p)
            if z is None:
                if is_init_partitioned(p):
                    p.data = gather_init_param(p).to(p.dtype).clone()
                    self.init_params.append(p)
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
            for p in self.init_params:
                if self.modifier_rank is not None:
                    if p._hds_part_world > 1:
                        g = p._hds_part_group
                        src = dist.get_global_rank(g, self.modifier_rank) if g is not None else self.modifier_rank
                        dist.broadcast(p.data, src, group=g)
                    flat = p.data.reshape(-1)
                    part = p._hds_part
                    pn = part.numel()
                    lo, hi = p._hds_part_rank * pn, min(flat.numel(), (p._hds_part_rank + 1) * pn)
                    part.zero_()
                    if hi > lo:
                        part[:hi - lo].copy_(flat[lo:hi])
                p.data = torch.empty(0, dtype=p.dtype, device=p.device)
            self.init_params = []
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
    """Declare that ``module``'s forward uses ``parameter`` of another module (reference
    partition_parameters.py register_external_parameter): the ZeRO-3 optimizer then gathers the parameter's unit
    around ``module``'s forward."""
    if not hasattr(module, "_external_params"):
        module._external_params = {}
    module._external_params[id(parameter)] = parameter


def unregister_external_parameter(module, parameter):
    if hasattr(module, "_external_params"):
        module._external_params.pop(id(parameter), None)


def _mark_leaf(m, flag):
    m._z3_leaf = bool(flag)
    for p in m.parameters():
        if flag:
            p.ds_z3_leaf_module = m
        else:
            p.__dict__.pop("ds_z3_leaf_module", None)


def set_z3_leaf_modules(model, leaf_module_classes):
    """Treat every instance of the given classes as ONE ZeRO-3 fetch unit (reference utils/z3_leaf_module.py). Must
    run before ``deepspeed.initialize`` builds the units. Returns the marked instances."""
    cur = tuple(getattr(model, "_z3_leaf_modules", ()))
    model._z3_leaf_modules = cur + tuple(c for c in leaf_module_classes if c not in cur)
    hit = [m for m in model.modules() if isinstance(m, tuple(leaf_module_classes))]
    for m in hit:
        _mark_leaf(m, True)
    return hit


def unset_z3_leaf_modules(model, leaf_module_classes):
    """Undo ``set_z3_leaf_modules`` for these classes. Returns the unmarked instances."""
    drop = tuple(leaf_module_classes)
    model._z3_leaf_modules = tuple(c for c in getattr(model, "_z3_leaf_modules", ()) if c not in drop)
    hit = [m for m in model.modules() if isinstance(m, drop)]
    for m in hit:
        _mark_leaf(m, False)
    return hit


def set_z3_leaf_module(model, flag):
    """Mark / unmark ONE module instance as a ZeRO-3 leaf (fetched as one unit)."""
    _mark_leaf(model, flag)


def z3_leaf_module(model):
    """Is this module a ZeRO-3 leaf (by instance mark or by one of its root's leaf classes)?"""
    return bool(getattr(model, "_z3_leaf", False))


def z3_leaf_parameter(param):
    """Does this parameter belong to a ZeRO-3 leaf module?"""
    return getattr(param, "ds_z3_leaf_module", None) is not None


def get_z3_leaf_modules(model):
    classes = tuple(getattr(model, "_z3_leaf_modules", ()))
    return [m for m in model.modules() if (classes and isinstance(m, classes)) or getattr(m, "_z3_leaf", False)]
