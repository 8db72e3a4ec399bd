"""Universal checkpoints: world-size independent per-parameter files, and re-sharded loading.

Layout (identical to the reference's, checkpoint/ds_to_universal.py:272-346,410-428)::

    <out>/zero/<param name>/fp32.pt, exp_avg.pt, exp_avg_sq.pt [, step.pt]
    <out>/zero/optimizer_state.pt          # non-sharded optimizer state + param_groups
    <out>/mp_rank_XX_model_states.pt       # model file(s) of the source checkpoint

ZeRO-0/1/2 sources give ``{"param": <full tensor>, "cat_dim": d, ...}`` files (plus ``step.pt``); ZeRO-3
sources without TP give the bare full tensor -- exactly what each reference loader expects
(universal_checkpoint.py:22-143 and stage3.py:2752-2827). Tensor-parallel slices are merged along the dims
in the source's ``universal_checkpoint_info``; loading cuts this rank's TP slice back out (``cat_dim``,
``sub_param_shape``, vocabulary padding) and then its data-parallel shard, so a run resumes on any number
of GPUs and any TP degree. Both file flavours are read here.
"""
import glob
import os
import shutil

import torch

from . import compat  # noqa: F401  (weights_only access to reference-pickled classes)
from .zero_to_fp32 import (_files_by_mp, _dp_rank, _load, _one_mp_rank, expert_global_name, merge_tp_slices)

_SHARDED = ("base_optimizer_state", "param_slice_mappings", "single_partition_of_fp32_groups", "fp32_flat_groups")


def _resolve(input_dir, tag):
    if tag is None and os.path.isfile(os.path.join(input_dir, "latest")):
        with open(os.path.join(input_dir, "latest")) as f:
            tag = f.read().strip()
    return os.path.join(input_dir, tag) if tag else input_dir


def _moment_keys(osd):
    stage = int(osd["zero_stage"])
    base = osd["optimizer_state_dict"] if stage == 3 else osd["base_optimizer_state"]
    keys = []
    for st in base.get("state", {}).values():
        for k, v in st.items():
            if torch.is_tensor(v) and v.dim() == 1 and k not in keys:
                keys.append(k)
    return keys


def _extract_job(job):
    """Worker: one (state key, TP rank) -> every parameter's merged-over-DP tensor, one temp file each."""
    key, mp, optim_files, model_file, model_files_all, tmp = job
    per_param = _one_mp_rank(optim_files, model_file, model_files_all, key=key)[0]
    for name, t in per_param.items():
        d = os.path.join(tmp, key, name)
        os.makedirs(d, exist_ok=True)
        torch.save(t.clone(), os.path.join(d, f"mp_{mp:02d}.pt"))
    return key, mp, len(per_param)


def _merge_job(job):
    """Worker: one (state key, parameter) -> its TP slices merged into the universal file."""
    key, name, mps, tmp, zdir, info, bare = job
    slices = [torch.load(os.path.join(tmp, key, name, f"mp_{mp:02d}.pt"), map_location="cpu", weights_only=True)
              for mp in mps]
    full, extra = merge_tp_slices(name, slices, info)
    d = os.path.join(zdir, name)
    os.makedirs(d, exist_ok=True)
    torch.save(full.clone() if bare else dict(extra, param=full), os.path.join(d, f"{key}.pt"))
    return name, key, tuple(full.shape), sum(t.numel() for t in slices)


def _run_pool(fn, jobs, workers):
    if workers <= 1 or len(jobs) <= 1:
        return [fn(j) for j in jobs]
    from concurrent.futures import ThreadPoolExecutor
    # threads: the jobs are torch.load / torch.save and tensor copies, which release the GIL; worker processes
    # would re-import torch per worker and (forked) can deadlock in an OpenMP pool the parent already used
    with ThreadPoolExecutor(max_workers=min(workers, len(jobs))) as ex:
        return list(ex.map(fn, jobs))


def ds_to_universal(input_dir, output_dir, tag=None, num_extract_workers=1, num_merge_workers=1,
                    keep_temp_folder=False, strict=True, inject_missing_state=False):
    """Convert ``<input_dir>/<tag>`` (a ZeRO checkpoint in the reference schema) into a universal checkpoint.

    Like the reference tool (checkpoint/ds_to_universal.py:469-540): (1) extraction -- one job per (state, TP
    rank) rebuilds every parameter from the DP shards into ``<out>/tmp`` -- runs on ``num_extract_workers``
    processes; (2) merging of the TP slices, one job per (state, parameter), on ``num_merge_workers`` processes
    (fewer: it holds whole parameters); (3) the non-sharded optimizer state. ``keep_temp_folder`` keeps ``tmp``;
    ``strict`` (default) fails on a parameter of the source's ``param_shapes`` that did not convert, whose element
    count changed in the merge, or that disagrees with the weights of the model states; ``inject_missing_state`` supplies a default ``universal_checkpoint_info`` to a
    ZeRO-1/2 source that lacks it (otherwise that is an error, as in the reference). Writes ``latest_universal``
    next to ``output_dir``."""
    ckpt_dir = _resolve(input_dir, tag)
    optim = _files_by_mp(ckpt_dir, "_optim_states.pt")
    models = _files_by_mp(ckpt_dir, "_model_states.pt")
    if not optim:
        raise FileNotFoundError(f"no *_optim_states.pt in {ckpt_dir}")
    osd0 = _load(optim[0][0])["optimizer_state_dict"]
    stage = int(osd0["zero_stage"])
    keys = ["fp32"] + _moment_keys(osd0)

    def model_file(mp):
        mf = models[mp]
        if stage <= 2:
            return [f for f in mf if os.path.basename(f).startswith("mp_rank_")][0]
        return [f for f in mf if _dp_rank(f) == 0][0]

    msd0 = _load(model_file(min(optim)))
    injected = None
    if "universal_checkpoint_info" not in msd0 and stage <= 2:
        if not inject_missing_state:
            raise ValueError(f"{model_file(min(optim))}: required 'universal_checkpoint_info' state is missing "
                             f"(the training client must record it, or pass inject_missing_state=True)")
        injected = {"universal_checkpoint_version": 0.2}
    info = msd0.get("universal_checkpoint_info") or injected or {}
    buffers = set(msd0.get("buffer_names") or [])
    zdir = os.path.join(output_dir, "zero")
    tmp = os.path.join(output_dir, "tmp")
    os.makedirs(zdir, exist_ok=True)
    # 1. extraction
    jobs = [(key, mp, optim[mp], model_file(mp), models[mp], tmp) for key in keys for mp in sorted(optim)]
    _run_pool(_extract_job, jobs, num_extract_workers)
    # 2. TP merge
    mps = sorted(optim)
    bare = stage == 3 and len(mps) == 1  # the reference stage-3 flavour: the bare tensor
    names = sorted(n for n in os.listdir(os.path.join(tmp, "fp32")) if n not in buffers)
    merged = _run_pool(_merge_job, [(key, n, mps, tmp, zdir, info, bare) for key in keys
                                    for n in names if os.path.isdir(os.path.join(tmp, key, n))], num_merge_workers)
    # 3. validity (strict) against the source's parameter list
    declared = set()
    for mp in mps:
        for d in (_load(model_file(mp)).get("param_shapes") or []):
            declared.update(d.keys())
    problems = []
    done = {(n, k) for n, k, _, _ in merged}
    for n in sorted(declared - buffers):
        for k in keys:
            if (n, k) not in done:
                problems.append(f"{n}: no {k} state converted")
    module = msd0.get("module") or {}
    for n, k, shape, n_slices in merged:
        numel = 1
        for x in shape:
            numel *= x
        if numel not in (n_slices, n_slices // max(1, len(mps))):
            problems.append(f"{n}/{k}: merged {numel} elements from {n_slices} in {len(mps)} TP slices")
        w = module.get(n)
        if k == "fp32" and torch.is_tensor(w) and numel not in (w.numel(), w.numel() * len(mps)):
            problems.append(f"{n}: {numel} elements converted, the model states hold {tuple(w.shape)}")
    if problems:
        msg = "universal conversion: " + "; ".join(problems[:10]) + (" ..." if len(problems) > 10 else "")
        if strict:
            raise ValueError(msg)
        from ..utils.logging import logger
        logger.warning(msg)
    if not keep_temp_folder:
        shutil.rmtree(tmp, ignore_errors=True)
    # global (non-sharded) optimizer state
    if stage == 3:
        gsd = dict(osd0)
        gsd.pop("fp32_flat_groups", None)
        base = gsd["optimizer_state_dict"]
        base = dict(base, state={g: {k: v for k, v in st.items() if not (torch.is_tensor(v) and v.dim() == 1)}
                                 for g, st in base.get("state", {}).items()})
        gsd["optimizer_state_dict"] = base
        gsd["param_groups"] = base.get("param_groups", [])
    else:
        gsd = {k: v for k, v in osd0.items() if k not in _SHARDED}
        gsd["param_groups"] = osd0["base_optimizer_state"].get("param_groups", [])
        steps = [st.get("step") for st in osd0["base_optimizer_state"].get("state", {}).values()]
        step = next((s for s in steps if s is not None), None)
        if step is not None:
            for name in os.listdir(zdir):
                if os.path.isdir(os.path.join(zdir, name)):
                    torch.save(step, os.path.join(zdir, name, "step.pt"))
    torch.save(gsd, os.path.join(zdir, "optimizer_state.pt"))
    # model files: one per TP rank under the world-size independent name
    for mp in mps:
        src = model_file(mp)
        dst = os.path.join(output_dir, f"mp_rank_{mp:02d}_model_states.pt")
        if injected is not None:
            sd = _load(src)
            sd["universal_checkpoint_info"] = injected
            torch.save(sd, dst)
        else:
            shutil.copyfile(src, dst)
    for f in glob.glob(os.path.join(ckpt_dir, "expp_rank_*")):
        shutil.copy2(f, output_dir)
    root, step_folder = os.path.split(os.path.normpath(output_dir))
    with open(os.path.join(root, "latest_universal"), "w") as f:
        f.write(step_folder)
    return output_dir


def _tp_slice(t, extra, target_shape, tp_rank, tp_world):
    """This TP rank's slice of a universal tensor (reference universal_checkpoint.py:43-124)."""
    if tuple(t.shape) == tuple(target_shape) or tp_world == 1:
        return t
    if extra.get("vocab_tensor", False):
        padded = target_shape[0] * tp_world
        if padded > t.shape[0]:
            t = torch.nn.functional.pad(t, (0, 0, 0, padded - t.shape[0]))
    sub = extra.get("sub_param_shape")
    if sub:
        sub = sub if isinstance(sub, dict) else vars(sub)
        dim = sub["partition_dim"]
        sizes = sub["shape"][dim]
        sizes = sizes if isinstance(sizes, (tuple, list)) else (sizes, )
        shape = [sum(d) if isinstance(d, (tuple, list)) else d for d in sub["shape"]]
        t = t.view(shape)
        chunks, off = [], 0
        for s in sizes:
            chunks.append(t.narrow(dim, off, s).chunk(tp_world, dim)[tp_rank])
            off += s
        return torch.cat(chunks, dim)
    dim = int(extra.get("cat_dim", 0))
    n_sub = int(extra.get("param_n_sub_params", 1))
    if n_sub > 1:
        return torch.cat([p.chunk(tp_world, dim)[tp_rank] for p in t.chunk(n_sub, dim)], dim)
    return t.chunk(tp_world, dim)[tp_rank]


def _read_universal(path):
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict):
        return obj["param"], {k: v for k, v in obj.items() if k != "param"}
    return obj, {}


def _universal_moment_keys(zdir):
    """Per-parameter optimizer-state file names (e.g. exp_avg, exp_avg_sq) of a universal checkpoint."""
    for name in sorted(os.listdir(zdir)):
        pdir = os.path.join(zdir, name)
        if not os.path.isdir(pdir) or not os.path.exists(os.path.join(pdir, "fp32.pt")):
            continue
        keys = []
        for f in sorted(os.listdir(pdir)):
            if not f.endswith(".pt") or f == "fp32.pt":
                continue
            t, _ = _read_universal(os.path.join(pdir, f))
            if torch.is_tensor(t) and t.numel() > 1:
                keys.append(f[:-3])
        return keys
    return []


def load_universal_into(zopt, universal_dir, load_optimizer_states=True):
    """Fill a (possibly differently sized / TP-sliced) ZeroOptimizer's shards from a universal checkpoint.

    Every rank reads only the parameter files overlapping its own shard. A missing ``fp32.pt`` is an error
    (never a silent zero-fill); missing moments are an error when ``load_optimizer_states``."""
    from ..utils import groups
    from ..utils.logging import logger
    zdir = os.path.join(universal_dir, "zero")
    if not os.path.isdir(zdir):
        raise FileNotFoundError(f"{universal_dir} is not a universal checkpoint (no zero/ folder)")
    tp_world, tp_rank = 1, 0
    if groups._State.topo is not None:
        tp_world, tp_rank = groups.get_model_parallel_world_size(), groups.get_model_parallel_rank()
    flats = zopt._ckpt_flats()
    if load_optimizer_states and zopt.kind == "generic":
        # a wrapped torch optimizer creates its state lazily: before its first step it has no moment flats, so take
        # the keys from the files and load into zero flats (as load_state_dict does)
        for k in _universal_moment_keys(zdir):
            if k not in flats:
                flats[k] = torch.zeros_like(flats["fp32"])
    keys = ["fp32"] + ([k for k in flats if k != "fp32"] if load_optimizer_states else [])
    with torch.no_grad():
        for u in zopt.units:
            lo, hi = u.rank * u.shard, (u.rank + 1) * u.shard
            for i, p in enumerate(u.params):
                a, b = max(lo, u.offsets[i]), min(hi, u.offsets[i] + u.numels[i])
                if a >= b:
                    continue
                name = zopt.param_names.get(id(p))
                if name is None:
                    raise ValueError(f"parameter {i} of ZeRO unit {u.name!r} has no name: cannot map it to a "
                                     "universal checkpoint file")
                j, nl = 0, int(getattr(p, "_hds_num_local", 1))
                stacked = getattr(p, "_hds_expert_stacked", False)
                if u.expert_key is not None:
                    j = zopt._ep_rank(u.expert_key)
                    if not stacked:
                        name = expert_global_name(name, j, nl)
                for key in keys:
                    f = os.path.join(zdir, name, f"{key}.pt")
                    if not os.path.exists(f):
                        raise FileNotFoundError(f"universal checkpoint has no {key!r} state for parameter {name!r} "
                                                f"({f})" + ("" if key == "fp32" else
                                                            "; pass load_optimizer_states=False to skip moments"))
                    t, extra = _read_universal(f)
                    if u.expert_key is not None and stacked:
                        t = t.view(-1, *u.shapes[i][1:])[j * nl:(j + 1) * nl]  # this EP rank's experts
                    if t.numel() != u.numels[i]:
                        t = _tp_slice(t, extra, u.shapes[i], tp_rank, tp_world)
                    if t.numel() != u.numels[i]:
                        raise ValueError(f"universal {key} of {name!r}: {t.numel()} elements, parameter has "
                                         f"{u.numels[i]} (shape {tuple(u.shapes[i])})")
                    t = t.reshape(-1).float()
                    dst = flats[key]
                    so = u.store_off + a - lo
                    dst[so:so + (b - a)].copy_(t[a - u.offsets[i]:b - u.offsets[i]])
        zopt._ckpt_commit(flats)
        zopt._master_to_lp()
    meta_f = os.path.join(zdir, "optimizer_state.pt")
    if os.path.exists(meta_f):
        meta = torch.load(meta_f, map_location="cpu", weights_only=True)
        pgs = meta.get("param_groups") or []
        if len(pgs) == len(zopt.param_groups):
            targets = list(zip(zopt.param_groups, pgs))
        else:
            targets = [(g, pgs[0]) for g in zopt.param_groups] if pgs else []
        for g, saved in targets:
            for k, v in saved.items():
                if k != "params":
                    g[k] = v
        ls = meta.get("loss_scaler")
        if isinstance(ls, dict):
            zopt.loss_scaler.load_state_dict(ls)
    else:
        logger.warning(f"{meta_f} missing: optimizer hyper-parameters / step count not restored")
    zopt._post_step_gather()
