#!/usr/bin/env python
"""Consolidate ZeRO (any stage, any data-parallel size) shards into one fp32 ``state_dict``.

Standalone (only needs torch), copied into every checkpoint directory like the reference's
utils/zero_to_fp32.py (:533 get_fp32_state_dict_from_zero_checkpoint, :598, :683 CLI)::

    python zero_to_fp32.py <checkpoint_dir> <output_file> [--tag global_step10]

Each ``*_optim_states.pt`` holds the rank's flat fp32 shard and the unit layout
{name, params, shapes, offsets, numels, shard, padded, store_off}. A unit's full flat buffer is the
rank-major concatenation of every rank's slice ``[store_off, store_off + shard)``; parameters are the
``[offset, offset + numel)`` ranges of that buffer.
"""
import argparse
import glob
import math
import os
import re

import torch


def _rank_of(path):
    m = re.search(r"zero_pp_rank_(\d+)_", os.path.basename(path))
    return int(m.group(1)) if m else 0


def _optim_files(ckpt_dir):
    files = glob.glob(os.path.join(ckpt_dir, "*_optim_states.pt"))
    files = [f for f in files if "expp_rank" not in f]
    if not files:
        raise FileNotFoundError(f"no *_optim_states.pt in {ckpt_dir}")
    by_mp = {}
    for f in files:
        mp = re.search(r"mp_rank_(\d+)", f)
        by_mp.setdefault(int(mp.group(1)) if mp else 0, []).append(f)
    return {mp: sorted(fs, key=_rank_of) for mp, fs in by_mp.items()}


def load_shards(ckpt_dir, states=("fp32", )):
    """Returns (layout, {state_name: [rank0 flat, rank1 flat, ...]}) for model-parallel rank 0."""
    files = _optim_files(ckpt_dir)[0]
    layout, out = None, {s: [] for s in states}
    for f in files:
        sd = torch.load(f, map_location="cpu", weights_only=True)["optimizer_state_dict"]
        layout = sd["layout"]
        for s in states:
            if s == "fp32":
                out[s].append(sd["fp32_flat_shard"].float())
            else:
                out[s].append(sd["optimizer_states"][s].float())
    return layout, out


_EXPERT_IDX = re.compile(r"(deepspeed_experts\.)(\d+)(\.)")


def expert_global_name(name, ep_rank, num_local):
    """Local expert parameter name on EP rank ``ep_rank`` -> name with the global expert index."""
    return _EXPERT_IDX.sub(lambda m: f"{m.group(1)}{int(m.group(2)) + ep_rank * num_local}{m.group(3)}", name,
                           count=1)


def unflatten(layout, flats):
    """flats: per-rank flat tensors (one per data-parallel rank) -> {param_name: full tensor}.

    Expert units (MoE, ``expert_group`` set) are sharded over their expert-data-parallel group: EP rank
    j's copy lives on data-parallel ranks ``j + ep_size * i``. Stacked expert weights ([E_local, ...]) are
    concatenated over EP ranks; per-expert modules get their global expert index in the name.
    """
    world = layout["world"]
    res = {}
    for u in layout["units"]:
        sh = u["shard"]
        if u.get("expert_group") is None:
            need = world
        else:
            need = u["ep_size"] * u["world"]
        if len(flats) < need:
            raise ValueError(f"checkpoint unit {u['name']} needs {need} shard files, found {len(flats)}")
        if u.get("expert_group") is None:
            full = torch.cat([flats[r][u["store_off"]:u["store_off"] + sh] for r in range(world)])
            for name, shape, off, n in zip(u["params"], u["shapes"], u["offsets"], u["numels"]):
                res[name] = full[off:off + n].view(shape).clone()
            continue
        P, W = u["ep_size"], u["world"]
        per_j = [torch.cat([flats[j + P * i][u["store_off"]:u["store_off"] + sh] for i in range(W)])
                 for j in range(P)]
        for k, (name, shape, off, n) in enumerate(zip(u["params"], u["shapes"], u["offsets"], u["numels"])):
            parts = [per_j[j][off:off + n].view(shape).clone() for j in range(P)]
            if u["expert_stacked"][k]:
                res[name] = torch.cat(parts, 0)
            else:
                for j in range(P):
                    res[expert_global_name(name, j, u["num_local"][k])] = parts[j]
    return res


def get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag=None, exclude_frozen_parameters=False):
    if tag is None:
        latest = os.path.join(checkpoint_dir, "latest")
        if os.path.isfile(latest):
            with open(latest) as f:
                tag = f.read().strip()
    ckpt_dir = os.path.join(checkpoint_dir, tag) if tag else checkpoint_dir
    layout, shards = load_shards(ckpt_dir)
    return unflatten(layout, shards["fp32"])


def convert_zero_checkpoint_to_fp32_state_dict(checkpoint_dir, output_file, tag=None, exclude_frozen_parameters=False):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag)
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
    a = ap.parse_args()
    sd = convert_zero_checkpoint_to_fp32_state_dict(a.checkpoint_dir, a.output_file, a.tag)
    print(f"saved {len(sd)} tensors ({sum(v.numel() for v in sd.values()) / 1e6:.1f}M params) to {a.output_file}")
