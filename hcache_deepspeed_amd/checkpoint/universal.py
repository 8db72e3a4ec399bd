"""Universal checkpoints: world-size independent per-parameter files, and re-sharded loading.

Reference parity: checkpoint/ds_to_universal.py (:112-198, :469 -- writes
``zero/<param_name>/{fp32,exp_avg,exp_avg_sq}.pt`` plus ``step``) and checkpoint/universal_checkpoint.py
``load_hp_checkpoint_state`` (:22-143). Here the conversion reads the flat-shard optimizer files
(see zero_to_fp32.py for the layout) and loading writes each new rank's shard of every unit from the
per-parameter fp32/moment tensors, so a run can resume on a different number of GPUs.
"""
import glob
import os

import torch

from .zero_to_fp32 import expert_global_name, load_shards, unflatten


def ds_to_universal(input_dir, output_dir, tag=None):
    """Convert ``<input_dir>/<tag>`` ZeRO shards into ``<output_dir>/zero/<param>/{fp32,exp_avg,exp_avg_sq}.pt``."""
    if tag is None and os.path.isfile(os.path.join(input_dir, "latest")):
        tag = open(os.path.join(input_dir, "latest")).read().strip()
    ckpt_dir = os.path.join(input_dir, tag) if tag else input_dir
    f0 = sorted(glob.glob(os.path.join(ckpt_dir, "*_optim_states.pt")))[0]
    sd0 = torch.load(f0, map_location="cpu", weights_only=True)["optimizer_state_dict"]
    names = ["fp32"] + list(sd0["optimizer_states"].keys())
    layout, shards = load_shards(ckpt_dir, states=tuple(names))
    zdir = os.path.join(output_dir, "zero")
    for s in names:
        full = unflatten(layout, shards[s])
        for pname, t in full.items():
            d = os.path.join(zdir, pname)
            os.makedirs(d, exist_ok=True)
            torch.save({"param": t}, os.path.join(d, f"{s}.pt"))
    step = sd0["param_groups"][0].get("step", 0) if sd0["param_groups"] else 0
    torch.save(torch.tensor(step), os.path.join(zdir, "optimizer_step.pt"))
    torch.save({"param_groups": sd0["param_groups"], "optimizer_kind": sd0["optimizer_kind"]},
               os.path.join(output_dir, "universal_meta.pt"))
    for mf in glob.glob(os.path.join(ckpt_dir, "*model_states.pt")):
        pass
    with open(os.path.join(output_dir, "latest_universal"), "w") as f:
        f.write(os.path.basename(output_dir.rstrip("/")))
    return output_dir


def load_universal_into(zopt, universal_dir, load_optimizer_states=True):
    """Fill a (possibly differently sized) ZeroOptimizer's shards from a universal checkpoint."""
    zdir = os.path.join(universal_dir, "zero")
    s = zopt.store
    states = ["fp32"] + (list(s.states.keys()) if load_optimizer_states else [])
    with torch.no_grad():
        for u in zopt.units:
            lo, hi = u.rank * u.shard, (u.rank + 1) * u.shard
            for st in states:
                dst = s.master if st == "fp32" else s.states[st]
                full = torch.zeros(u.padded, dtype=torch.float32)
                for i, p in enumerate(u.params):
                    name = zopt.param_names.get(id(p))
                    j, nl = 0, int(getattr(p, "_hds_num_local", 1))
                    if u.expert_key is not None:
                        j = zopt._ep_rank(u.expert_key)
                        if not getattr(p, "_hds_expert_stacked", False):
                            name = expert_global_name(name, j, nl)
                    f = os.path.join(zdir, name, f"{st}.pt")
                    if os.path.exists(f):
                        t = torch.load(f, map_location="cpu", weights_only=True)["param"]
                        if u.expert_key is not None and getattr(p, "_hds_expert_stacked", False):
                            t = t[j * nl:(j + 1) * nl]  # this EP rank's experts of the global stack
                        full[u.offsets[i]:u.offsets[i] + u.numels[i]] = t.reshape(-1).float()
                dst[u.store_off:u.store_off + u.shard].copy_(full[lo:hi].to(dst.device))
        s.lp.copy_(s.master)
    meta_f = os.path.join(universal_dir, "universal_meta.pt")
    if os.path.exists(meta_f):
        meta = torch.load(meta_f, map_location="cpu", weights_only=True)
        for g, saved in zip(zopt.param_groups, meta["param_groups"]):
            for k, v in saved.items():
                g[k] = v
    zopt._post_step_gather()
