"""DeepSpeed-format ZeRO optimizer state <-> this framework's flat-unit shard store.

The training-time layout (flat.py) is chosen for the hardware: one rank-major flat buffer per
transformer block so a gather is ONE all-gather and a gradient reduction ONE reduce-scatter. The
checkpoint layout is chosen for interoperability: it is the reference's, so the reference's
``zero_to_fp32.py`` / ``ds_to_universal.py`` read our files and we read the reference's.

Reference layouts ("ref groups" = one per optimizer param group, split by MoE expert group like
``split_params_into_different_moe_groups_for_optimizer``; params in param-group order):

* ZeRO-0/1/2 (stage_1_and_2.py:2156-2200, zero_to_fp32.py:252-322): the group's params are
  concatenated (no per-param padding), padded to a multiple of ``2 * world`` and cut into ``world``
  equal partitions ``P``. Rank r saves ``single_partition_of_fp32_groups[g]`` = its partition without
  the trailing padding, the moments in ``base_optimizer_state['state'][g]`` and, per param it touches,
  ``param_slice_mappings[g][name] = fragment_address(numel, start)``.
* ZeRO-3 (stage3.py:2544-2560, zero_to_fp32.py:437-487): every param is split on its own into
  ``ceil(numel / world)``-element partitions; rank r's ``fp32_flat_groups[g]`` is the concatenation of its
  partition of every param (zero padded), moments in ``optimizer_state_dict['state'][g]``.

Moving between the two layouts is a per-unit collective: saving all-gathers a unit's fp32/moment shard
and every rank copies out the ranges its reference partition covers; loading scatters each rank's
reference partition into a zero unit buffer and reduce-scatters it (the ranges are disjoint, so the
sum is exact) straight into the rank's shard. One unit is resident at a time.
"""
import math
from collections import OrderedDict

import torch

from ... import comm as dist
from ...utils.tensor_fragment import fragment_address

FP32 = "fp32"


class RefGroup:
    __slots__ = ("param_group", "params", "world", "rank", "part", "padding", "places", "mappings", "dp_group")

    def __init__(self, param_group, params, world, rank, dp_group):
        self.param_group = param_group
        self.params = params  # [(name, param, unit, index)]
        self.world, self.rank, self.dp_group = world, rank, dp_group
        self.part = 0
        self.padding = 0
        self.places = []  # [(unit, unit_offset, numel, partition_offset)] for THIS rank
        self.mappings = OrderedDict()


def _name(z, p):
    n = z.param_names.get(id(p))
    if n is None:
        raise ValueError("ZeRO checkpoint: a parameter managed by the optimizer has no name (was the model "
                         "modified after deepspeed.initialize?)")
    return n


def ref_groups(z, order=None):
    """Build the reference layout for optimizer ``z`` (a ZeroOptimizer).

    ``order``: optional list (one per ref group) of parameter names -- the order a checkpoint was written
    in (its ``param_shapes``); default is the optimizer's own param-group order."""
    if order is None:
        raw = []
        for gi, g in enumerate(z.param_groups):
            by = OrderedDict()
            for p in g["params"]:
                u, i = z.param_to_unit[id(p)]
                by.setdefault(u.expert_key, []).append((_name(z, p), p, u, i))
            raw.extend((gi, lst) for lst in by.values())
    else:
        byname, gi_of = {}, {}
        for gi, g in enumerate(z.param_groups):
            for p in g["params"]:
                byname[_name(z, p)] = p
                gi_of[id(p)] = gi
        raw = []
        for names in order:
            lst = []
            for n in names:
                if n not in byname:
                    raise KeyError(f"checkpoint parameter {n!r} does not exist in this model's optimizer")
                p = byname[n]
                u, i = z.param_to_unit[id(p)]
                lst.append((n, p, u, i))
            if lst:
                raw.append((gi_of[id(lst[0][1])], lst))
    out = []
    for gi, lst in raw:
        u0 = lst[0][2]
        assert all(t[2].world == u0.world for t in lst), "a ref group must live on one data-parallel group"
        g = RefGroup(gi, lst, u0.world, u0.rank, u0.dp_group)
        W, r = g.world, g.rank
        if z.stage == 3:
            base = 0
            for name, p, u, i in lst:
                n = u.numels[i]
                pn = math.ceil(n / W)
                lo, hi = r * pn, min(n, (r + 1) * pn)
                if hi > lo:
                    g.places.append((u, u.offsets[i] + lo, hi - lo, base))
                base += pn
            g.part = base
        else:
            total = sum(t[2].numels[t[3]] for t in lst)
            align = 2 * W
            padded = align * math.ceil(total / align)
            P = padded // W
            lo_r, hi_r = r * P, (r + 1) * P
            base = 0
            for name, p, u, i in lst:
                n = u.numels[i]
                a, b = max(base, lo_r), min(base + n, hi_r)
                if a < b:
                    g.places.append((u, u.offsets[i] + a - base, b - a, a - lo_r))
                    g.mappings[name] = fragment_address(numel=b - a, start=a - lo_r)
                base += n
            g.part = P
            g.padding = (padded - total) if r == W - 1 else 0
        out.append(g)
    return out


def param_shapes(groups):
    """``param_shapes`` for the model-state file: one OrderedDict(name -> torch.Size) per ref group."""
    return [OrderedDict((n, torch.Size(u.shapes[i])) for n, _, u, i in g.params) for g in groups]


def _unit_places(groups):
    by = {}
    for gidx, g in enumerate(groups):
        for u, a, n, d in g.places:
            by.setdefault(u.uid, []).append((gidx, a, n, d))
    return by


def export_partitions(z, flats, groups):
    """flats: {key: store-sized fp32 tensor (any device)} -> {key: [per ref group CPU partition]}."""
    places = _unit_places(groups)
    out = {k: [torch.zeros(g.part, dtype=torch.float32) for g in groups] for k in flats}
    for u in z.units:
        pl = places.get(u.uid, [])
        if u.world == 1 and not pl:
            continue
        for k, flat in flats.items():
            shard = flat[u.store_off:u.store_off + u.shard]
            if u.world > 1:
                full = torch.empty(u.padded, dtype=torch.float32, device=z.device)
                dist.all_gather_into_tensor(full, shard.to(z.device, torch.float32), group=u.dp_group)
            else:
                full = shard
            for gidx, a, n, d in pl:
                out[k][gidx][d:d + n].copy_(full[a:a + n])
    return out


def import_partitions(z, parts, groups, dst_flats):
    """parts: {key: [per ref group partition]} (this rank's reference partitions) -> write every unit's shard of
    ``dst_flats[key]`` (store-sized tensors, any device). Collective over each unit's data-parallel group."""
    places = _unit_places(groups)
    for u in z.units:
        pl = places.get(u.uid, [])
        if u.world == 1 and not pl:
            continue
        for k, dst in dst_flats.items():
            src = parts[k]
            contrib = torch.zeros(u.padded, dtype=torch.float32, device=z.device)
            for gidx, a, n, d in pl:
                contrib[a:a + n].copy_(src[gidx][d:d + n])
            if u.world > 1:
                mine = torch.empty(u.shard, dtype=torch.float32, device=z.device)
                dist.reduce_scatter_tensor(mine, contrib, group=u.dp_group)
            else:
                mine = contrib[:u.shard]
            dst[u.store_off:u.store_off + u.shard].copy_(mine)


def _hp(group):
    return {k: v for k, v in group.items() if k != "params"}


def build_state_dict(z, flats, scalars):
    """The optimizer half of a ZeRO checkpoint in the reference schema.

    flats: {"fp32": master, <state key>: tensor} store-sized; scalars: {param_group index: {"step": int}}."""
    groups = ref_groups(z)
    parts = export_partitions(z, flats, groups)
    moments = [k for k in flats if k != FP32]
    state = {}
    for gidx, g in enumerate(groups):
        st = dict(scalars.get(g.param_group, {}))
        for k in moments:
            st[k] = parts[k][gidx]
        state[gidx] = st
    base = {"state": state, "param_groups": [dict(_hp(z.param_groups[g.param_group]), params=[gidx])
                                               for gidx, g in enumerate(groups)]}
    sd = OrderedDict()
    sd["loss_scaler"] = z.loss_scaler.state_dict()
    sd["dynamic_loss_scale"] = z.loss_scaler.dynamic
    sd["overflow"] = z.overflow
    sd["clip_grad"] = z.clip_grad
    if z.stage == 3:
        sd["zero_stage"] = 3
        worlds = [g.world for g in groups] or [1]
        sd["partition_count"] = worlds[0] if len(set(worlds)) == 1 else worlds
        sd["optimizer_state_dict"] = base
        sd["fp32_flat_groups"] = parts[FP32]
    else:
        sd["zero_stage"] = z.stage
        sd["base_optimizer_state"] = base
        sd["single_partition_of_fp32_groups"] = [t[:g.part - g.padding] for t, g in zip(parts[FP32], groups)]
        sd["group_paddings"] = [g.padding for g in groups]
        sd["partition_count"] = [g.world for g in groups]
        sd["param_slice_mappings"] = [g.mappings for g in groups]
    from ...version import __version__
    sd["ds_version"] = __version__
    # name order of every ref group (also recoverable from the model file's param_shapes)
    sd["hds_param_order"] = [[n for n, _, _, _ in g.params] for g in groups]
    sd["hds_optimizer_kind"] = z.kind
    metas = []
    for g in groups:
        key = g.params[0][2].expert_key
        if key is None:
            metas.append(None)
            continue
        metas.append({"expert_group": key, "ep_size": z._ep_size(key), "ep_rank": z._ep_rank(key),
                      "expert_stacked": [bool(getattr(p, "_hds_expert_stacked", False)) for _, p, _, _ in g.params],
                      "num_local": [int(getattr(p, "_hds_num_local", 1)) for _, p, _, _ in g.params]})
    sd["hds_group_meta"] = metas
    return sd


def _split_like(flat, groups):
    """Cut one rank's concatenated stage-3 sub-group flats into this model's per-group partitions. A shortfall is
    accepted only up to the alignment padding a writer may leave off the tail (2 * world elements per group); a
    larger one means a mismatched or truncated checkpoint and raises instead of loading zeros."""
    total = sum(g.part for g in groups)
    slack = sum(2 * g.world for g in groups)
    if flat.numel() + slack < total:
        raise ValueError(f"stage-3 sub-group flats hold {flat.numel()} elements per rank, this model needs {total}")
    out, off = [], 0
    for g in groups:
        n = min(g.part, max(0, flat.numel() - off))
        t = flat.narrow(0, off, n)
        out.append(t if n == g.part else torch.cat([t, t.new_zeros(g.part - n)]))
        off += g.part
    if off < flat.numel() and bool(flat[off:].abs().sum() > 0):
        raise ValueError(f"stage-3 sub-group flats hold {flat.numel()} elements per rank, this model {off}")
    return out


def _regroup_stage3(fp32, base, groups):
    """Sub-group flats (any count) -> one partition per ref group of this optimizer, for fp32 and every moment."""
    fp32 = _split_like(torch.cat([t.float().view(-1) for t in fp32]), groups)
    st = base.get("state", {})
    keys = sorted(st, key=lambda k: int(k))
    new_st = {}
    if keys:
        first = st[keys[0]]
        merged = {}
        for k, v in first.items():
            if torch.is_tensor(v) and v.dim() == 1:
                merged[k] = _split_like(torch.cat([st[i][k].float().view(-1) for i in keys]), groups)
        for gidx in range(len(groups)):
            new_st[gidx] = {k: (merged[k][gidx] if k in merged else v) for k, v in first.items()}
    base = dict(base)
    base["state"] = new_st
    return fp32, base


def read_state_dict(z, sd, order=None):
    """Parse a reference-schema optimizer state (ours or the reference's) for optimizer ``z``.

    Returns (groups, parts {key: [partition per ref group]}, scalars per ref group, param_groups hp)."""
    if order is None:
        order = sd.get("hds_param_order")
    if order is None:
        raise ValueError("optimizer checkpoint has no parameter order: pass the model file's param_shapes")
    groups = ref_groups(z, order)
    stage = int(sd.get("zero_stage", z.stage))
    if (stage == 3) != (z.stage == 3):
        raise ValueError(f"checkpoint is ZeRO stage {stage}, engine runs stage {z.stage}: convert it with "
                         "ds_to_universal and load with checkpoint.load_universal")
    if stage == 3:
        fp32 = sd["fp32_flat_groups"]
        base = sd["optimizer_state_dict"]
    else:
        fp32 = sd["single_partition_of_fp32_groups"]
        base = sd["base_optimizer_state"]
    pc = sd.get("partition_count")
    if stage == 3 and len(fp32) != len(groups):
        # the reference's stage 3 writes one flat per sub-group (sub_group_size, stage3.py:2082-2144), not one per
        # param group; params run back to back across them (reference utils/zero_to_fp32.py:437-477)
        fp32, base = _regroup_stage3(fp32, base, groups)
        pc = pc if not isinstance(pc, list) else pc[0]
    pcs = pc if isinstance(pc, list) else [pc] * len(groups)
    if len(fp32) != len(groups):
        raise ValueError(f"checkpoint has {len(fp32)} flat groups, this optimizer {len(groups)}")
    for g, w in zip(groups, pcs):
        if w is not None and int(w) != g.world:
            raise ValueError(f"checkpoint partition count {w} != data-parallel size {g.world}: load it through a "
                             "universal checkpoint (ds_to_universal + checkpoint.load_universal)")
    parts = {FP32: [t.float() for t in fp32]}
    scalars = []
    st = base.get("state", {})
    for gidx in range(len(groups)):
        s = st.get(gidx, {})
        sc = {}
        for k, v in s.items():
            if torch.is_tensor(v) and v.dim() == 1:
                parts.setdefault(k, [None] * len(groups))[gidx] = v.float()
            else:
                sc[k] = v.item() if torch.is_tensor(v) else v
        scalars.append(sc)
    # single_partition_of_fp32_groups is saved without the trailing padding: widen to the partition size
    for k, lst in parts.items():
        for gidx, (t, g) in enumerate(zip(lst, groups)):
            if t is None:
                continue
            if t.numel() < g.part:
                lst[gidx] = torch.cat([t, t.new_zeros(g.part - t.numel())])
    hps = [{k: v for k, v in pg.items() if k != "params"} for pg in base.get("param_groups", [])]
    return groups, parts, scalars, hps
