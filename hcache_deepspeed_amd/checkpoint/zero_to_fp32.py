#!/usr/bin/env python
"""Consolidate a ZeRO checkpoint (any stage, any data-parallel size) into one fp32 ``state_dict``.

Standalone (needs only torch): it is copied into every checkpoint directory like the reference's
utils/zero_to_fp32.py (API :533 ``get_fp32_state_dict_from_zero_checkpoint``, :598
``convert_zero_checkpoint_to_fp32_state_dict``, :683 ``load_state_dict_from_zero_checkpoint``)::

    python zero_to_fp32.py <checkpoint_dir> <output_file> [--tag global_step10]

Files follow the reference schema (see runtime/zero/ds_state.py), so the reconstruction protocol is the
reference's:

* ZeRO-0/1/2: concatenate every rank's ``single_partition_of_fp32_groups[g]``; params of group g are
  consecutive ``numel``-element runs in ``param_shapes[g]`` order (the tail is 2*world alignment padding).
* ZeRO-3: param p's value is the concatenation over ranks of its ``ceil(numel / world)``-element slice
  of ``fp32_flat_groups``; slices are laid out back to back in ``param_shapes`` order.

Beyond the reference: MoE expert groups (sharded over their expert-data-parallel group; ``hds_group_meta``
says which files hold which expert-parallel rank) and tensor parallelism (one file set per
``mp_rank_XX``, merged along the dims recorded in ``universal_checkpoint_info``). Everything is read with
``torch.load(weights_only=True)``; the reference's pickled helper classes are mapped to local stand-ins.
"""
import argparse
import glob
import math
import os
import re
from collections import OrderedDict
from dataclasses import dataclass
from enum import Enum
from typing import List, Tuple, Union

import torch


@dataclass
class _FragmentAddress:
    numel: int
    start: int


class _ZeroStage(int, Enum):
    disabled = 0
    optimizer_states = 1
    gradients = 2
    weights = 3
    max_stage = 3


@dataclass
class _SubparamShape:
    patterns: List[str]
    shape: Tuple[Union[Tuple[int], int]]
    partition_dim: int


class _LossScalerState:
    pass


def _register_safe_globals():
    allowed = [(_FragmentAddress, "deepspeed.utils.tensor_fragment.fragment_address"),
               (_FragmentAddress, "hcache_deepspeed_amd.utils.tensor_fragment.fragment_address"),
               (_ZeroStage, "deepspeed.runtime.zero.config.ZeroStageEnum"),
               (_SubparamShape, "deepspeed.checkpoint.universal_checkpoint.SubparamShape"),
               (_SubparamShape, "hcache_deepspeed_amd.checkpoint.compat.SubparamShape"),
               (_LossScalerState, "deepspeed.runtime.fp16.loss_scaler.LossScaler"),
               (_LossScalerState, "deepspeed.runtime.fp16.loss_scaler.DynamicLossScaler")]
    try:
        torch.serialization.add_safe_globals(allowed)
    except (AttributeError, TypeError):  # torch without (fn, name) pairs: our own files need none of these
        pass


_register_safe_globals()


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def _natural(text):
    return [int(c) if c.isdigit() else c for c in re.split(r"(\d+)", text)]


def _dp_rank(path):
    m = re.search(r"zero_pp_rank_(\d+)_", os.path.basename(path))
    return int(m.group(1)) if m else 0


def _mp_rank(path):
    m = re.search(r"mp_rank_(\d+)", os.path.basename(path))
    return int(m.group(1)) if m else 0


def _files_by_mp(ckpt_dir, suffix):
    files = [f for f in glob.glob(os.path.join(ckpt_dir, f"*{suffix}")) if "expp_rank" not in os.path.basename(f)]
    by = OrderedDict()
    for f in sorted(files, key=_natural):
        by.setdefault(_mp_rank(f), []).append(f)
    return {m: sorted(fs, key=_dp_rank) for m, fs in by.items()}


def _numel(shape):
    return int(math.prod(shape))


def _reconstruct(stage, shapes, parts, exact=True):
    """shapes: OrderedDict name -> shape of one flat group; parts: that group's partition on each rank, in rank
    order -> OrderedDict name -> fp32 tensor."""
    out = OrderedDict()
    if stage <= 2:
        full = torch.cat([p.float() for p in parts]) if len(parts) > 1 else parts[0].float()
        off = 0
        for name, shape in shapes.items():
            n = _numel(shape)
            out[name] = full.narrow(0, off, n).view(tuple(shape)).clone()
            off += n
        align = 2 * len(parts)
        if align * math.ceil(off / align) != align * math.ceil(full.numel() / align):
            raise ValueError(f"consumed {off} of {full.numel()} elements: checkpoint / param_shapes mismatch")
        return out
    W = len(parts)
    off = 0
    for name, shape in shapes.items():
        n = _numel(shape)
        pn = math.ceil(n / W)
        out[name] = torch.cat([p.narrow(0, off, pn).float() for p in parts]).narrow(0, 0, n).view(tuple(shape)).clone()
        off += pn
    if off > parts[0].numel() or (exact and off != parts[0].numel()):
        raise ValueError(f"consumed {off} of {parts[0].numel()} elements per rank: checkpoint / param_shapes mismatch")
    return out


_EXPERT_IDX = re.compile(r"(deepspeed_experts\.)(\d+)(\.)")


def expert_global_name(name, ep_rank, num_local):
    """Local expert parameter name on EP rank ``ep_rank`` -> name with the global expert index."""
    return _EXPERT_IDX.sub(lambda m: f"{m.group(1)}{int(m.group(2)) + ep_rank * num_local}{m.group(3)}", name,
                           count=1)


def _partition(osd, g, key):
    """Flat group ``g``'s partition of ``key`` ("fp32" master weights or an optimizer moment) in one rank's file."""
    stage = int(osd["zero_stage"])
    if key == "fp32":
        return (osd["fp32_flat_groups"] if stage == 3 else osd["single_partition_of_fp32_groups"])[g]
    base = osd["optimizer_state_dict"] if stage == 3 else osd["base_optimizer_state"]
    st = base["state"]
    return st[g][key] if g in st else st[str(g)][key]


def _one_mp_rank(optim_files, model_file, model_files_all, key="fp32"):
    sds = [_load(f)["optimizer_state_dict"] for f in optim_files]
    if key == "fp32":
        for sd in sds:
            sd.pop("optimizer_state_dict", None)  # moments are not needed here
            sd.pop("base_optimizer_state", None)
    stage = int(sds[0]["zero_stage"])
    msd = _load(model_file)
    shapes = msd["param_shapes"]
    metas = sds[0].get("hds_group_meta") or [None] * len(shapes)
    pcs = sds[0]["partition_count"]
    pcs = pcs if isinstance(pcs, list) else [pcs] * max(len(shapes), 1)
    by_rank = {_dp_rank(f): sd for f, sd in zip(optim_files, sds)}
    state = OrderedDict()
    buffers = set(msd.get("buffer_names") or [])
    for n, t in (msd.get("module") or {}).items():
        if n in buffers and key == "fp32":
            state[n] = t.float()
    if stage == 3 and all(m is None for m in metas) and len(by_rank[0]["fp32_flat_groups"]) != len(shapes):
        # the reference's stage 3 writes one flat per sub-group (sub_group_size), not per param group: walk the
        # merged param_shapes over each rank's concatenated sub-group flats (reference zero_to_fp32.py:437-477)
        W = int(pcs[0])
        if len(by_rank) < W:
            raise ValueError(f"expected {W} '*_optim_states.pt' files, found {len(by_rank)}")
        merged = OrderedDict((n, s) for d in shapes for n, s in d.items())
        parts = []
        for r in range(W):
            n_sub = len(by_rank[r]["fp32_flat_groups"])
            parts.append(torch.cat([_partition(by_rank[r], i, key).view(-1) for i in range(n_sub)]))
        state.update(_reconstruct(stage, merged, parts))  # exact, as the reference's sanity check (:481-485)
        shapes, metas = [], []
    for g, (shp, meta) in enumerate(zip(shapes, metas)):
        W = int(pcs[g])
        if meta is None or meta.get("expert_group") is None:
            if stage > 0 and len(by_rank) < W:
                raise ValueError(f"expected {W} '*_optim_states.pt' files, found {len(by_rank)}")
            parts = [_partition(by_rank[r], g, key) for r in range(W)]
            state.update(_reconstruct(stage, shp, parts))
            continue
        P = int(meta["ep_size"])
        per_j = []
        for j in range(P):
            ranks = [j + P * i for i in range(W)] if stage > 0 else [j]
            missing = [r for r in ranks if r not in by_rank]
            if missing:
                raise ValueError(f"expert group {meta['expert_group']}: missing optimizer files of ranks {missing}")
            per_j.append(_reconstruct(stage, shp, [_partition(by_rank[r], g, key) for r in ranks]))
        for k, name in enumerate(shp):
            if meta["expert_stacked"][k]:
                state[name] = torch.cat([per_j[j][name] for j in range(P)], 0)
            else:
                for j in range(P):
                    state[expert_global_name(name, j, meta["num_local"][k])] = per_j[j][name]
    frozen = msd.get("frozen_param_shapes")
    if frozen and key == "fp32":
        if stage == 3:
            frag_sds = [_load(f) for f in model_files_all]
            for name, shape in frozen.items():
                n = _numel(shape)
                state[name] = torch.cat([fs["frozen_param_fragments"][name].float() for fs in frag_sds]
                                        ).narrow(0, 0, n).view(tuple(shape)).clone()
        else:
            for name in frozen:
                state[name] = msd["frozen_param_fragments"][name].float()
    for alias, owner in (msd.get("shared_params") or {}).items():
        if owner in state:
            state[alias] = state[owner]
    return state, msd


def merge_tp_slices(name, slices, info):
    """Full tensor from per-TP-rank slices, using ``universal_checkpoint_info`` (reference ds_to_universal.py:232
    merge_tp_slices). Returns (tensor, extra keys for a universal checkpoint file)."""
    if len(slices) == 1:
        return slices[0], {"cat_dim": 0}

    def match(key):
        return any(re.match(p, name) for p in info.get(key, []) or [])

    if match("tp_replicated_parameter_patterns"):
        return slices[0], {}
    if match("parameter_to_average_patterns"):
        return sum(slices) / len(slices), {}
    for sp in info.get("parameter_with_sub_params", []) or []:
        sp = sp if isinstance(sp, dict) else vars(sp)
        if any(re.match(p, name) for p in sp["patterns"]):
            dim = sp["partition_dim"]
            sizes = sp["shape"][dim]
            sizes = sizes if isinstance(sizes, (tuple, list)) else (sizes, )
            tp = len(slices)
            chunks, off = [], 0
            for s in sizes:
                chunks.append(torch.cat([t.narrow(dim, off, s // tp) for t in slices], dim))
                off += s // tp
            return torch.cat(chunks, dim), {"sub_param_shape": sp}
    if match("parameter_with_2_sub_params_cat_dim_0"):
        halves = [t.chunk(2, 0) for t in slices]
        return torch.cat([torch.cat([h[0] for h in halves]), torch.cat([h[1] for h in halves])]), \
            {"cat_dim": 0, "param_n_sub_params": 2}
    dim = 1 if match("parameter_with_row_parallelism_patterns") else 0
    return torch.cat(slices, dim), {"cat_dim": dim}


def _resolve(checkpoint_dir, tag):
    if tag is None:
        latest = os.path.join(checkpoint_dir, "latest")
        if os.path.isfile(latest):
            with open(latest) as f:
                tag = f.read().strip()
    return os.path.join(checkpoint_dir, tag) if tag else checkpoint_dir


def get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag=None, exclude_frozen_parameters=False):
    ckpt_dir = _resolve(checkpoint_dir, tag)
    optim = _files_by_mp(ckpt_dir, "_optim_states.pt")
    if not optim:
        raise FileNotFoundError(f"no *_optim_states.pt in {ckpt_dir}")
    models = _files_by_mp(ckpt_dir, "_model_states.pt")
    per_mp = []
    for mp, files in optim.items():
        stage = int(_load(files[0])["optimizer_state_dict"]["zero_stage"])
        mfiles = models[mp]
        if stage <= 2:
            mfile = [f for f in mfiles if os.path.basename(f).startswith("mp_rank_")][0]
        else:
            mfile = [f for f in mfiles if _dp_rank(f) == 0][0]
        state, msd = _one_mp_rank(files, mfile, mfiles)
        if exclude_frozen_parameters:
            for name in (msd.get("frozen_param_shapes") or {}):
                state.pop(name, None)
        per_mp.append((state, msd))
    if len(per_mp) == 1:
        return per_mp[0][0]
    info = per_mp[0][1].get("universal_checkpoint_info") or {}
    merged = OrderedDict()
    for name in per_mp[0][0]:
        merged[name] = merge_tp_slices(name, [s[name] for s, _ in per_mp], info)[0]
    return merged


def convert_zero_checkpoint_to_fp32_state_dict(checkpoint_dir, output_file, tag=None, exclude_frozen_parameters=False):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag, exclude_frozen_parameters)
    torch.save(sd, output_file)
    return sd


def load_state_dict_from_zero_checkpoint(model, checkpoint_dir, tag=None):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag)
    model.load_state_dict(sd, strict=False)
    return model


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("checkpoint_dir")
    ap.add_argument("output_file")
    ap.add_argument("-t", "--tag", default=None)
    ap.add_argument("--exclude_frozen_parameters", action="store_true")
    a = ap.parse_args()
    sd = convert_zero_checkpoint_to_fp32_state_dict(a.checkpoint_dir, a.output_file, a.tag,
                                                    a.exclude_frozen_parameters)
    print(f"saved {len(sd)} tensors ({sum(v.numel() for v in sd.values()) / 1e6:.1f}M params) to {a.output_file}")
