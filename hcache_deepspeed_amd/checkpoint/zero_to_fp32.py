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


def unflatten(layout, flats):
    """flats: per-rank flat tensors (one per data-parallel rank) -> {param_name: full tensor}."""
    world = layout["world"]
    if len(flats) < world:
        raise ValueError(f"checkpoint was written by {world} ranks, found {len(flats)} shard files")
    res = {}
    for u in layout["units"]:
        sh = u["shard"]
        full = torch.cat([flats[r][u["store_off"]:u["store_off"] + sh] for r in range(world)])
        for name, shape, off, n in zip(u["params"], u["shapes"], u["offsets"], u["numels"]):
            res[name] = full[off:off + n].view(shape).clone()
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
