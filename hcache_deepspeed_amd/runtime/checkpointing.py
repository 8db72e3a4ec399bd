"""Engine checkpoint save/load with the DeepSpeed directory layout and file names.

Reference parity: runtime/engine.py save_checkpoint :3274 / load_checkpoint :2928, file names
:2857-2917 (``mp_rank_XX_model_states.pt``, ``zero_pp_rank_{dp}_mp_rank_{mp:02d}_model_states.pt``,
``[bf16_]zero_pp_rank_{dp}_mp_rank_{mp:02d}_optim_states.pt``), the ``latest`` tag file (:3357-3359), the
model-state keys (:3525-3546), and the copy of ``zero_to_fp32.py`` into the checkpoint dir (:3674-3691).

File CONTENTS follow the reference schema too (runtime/zero/ds_state.py): ZeRO-1/2 optimizer files hold
``single_partition_of_fp32_groups`` / ``base_optimizer_state`` / ``param_slice_mappings`` / ``group_paddings`` /
``partition_count``, ZeRO-3 files ``fp32_flat_groups`` / ``optimizer_state_dict``, and model files
``param_shapes`` / ``buffer_names`` / ``shared_params`` / ``frozen_param_*`` / ``universal_checkpoint_info``, so
the reference's ``zero_to_fp32.py`` and ``ds_to_universal.py`` reconstruction protocols apply unchanged.

Saves are asynchronous when ``checkpoint.async_save`` is set: background threads write the files while
training continues, and ``latest`` moves only after EVERY rank's files are complete (per-rank commit
markers, atomic rename), so a crash mid-save resumes from the previous tag.
"""
import math
import os
import re
import shutil
import threading
from collections import OrderedDict

import torch

from .. import comm as dist
from ..utils import groups
from ..utils.logging import log_dist, logger
from ..version import __version__

_ASYNC_THREADS = []


def _mp_rank():
    return groups.get_model_parallel_rank() if groups._State.topo is not None else 0


def _ckpt_name(engine, save_dir, tag):
    mp = _mp_rank()
    if engine.zero_optimization_stage() == 3:
        dp = dist.get_rank(engine.dp_group)
        return os.path.join(save_dir, str(tag), f"zero_pp_rank_{dp}_mp_rank_{mp:02d}_model_states.pt")
    return os.path.join(save_dir, str(tag), f"mp_rank_{mp:02d}_model_states.pt")


def _optim_name(engine, save_dir, tag):
    mp = _mp_rank()
    dp = dist.get_rank(engine.dp_group)
    prefix = "bf16_" if engine.bfloat16_enabled() else ""
    return os.path.join(save_dir, str(tag), f"{prefix}zero_pp_rank_{dp}_mp_rank_{mp:02d}_optim_states.pt")


def _max_ep(zopt):
    return max(zopt._ep_size(u.expert_key) for u in zopt.expert_units)


def _expert_name(save_dir, tag, ep_rank):
    return os.path.join(save_dir, str(tag), f"expp_rank_{ep_rank}_mp_rank_{_mp_rank():02d}_model_states.pt")


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return type(obj)((k, _to_cpu(v)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def _write(obj, path, async_save):
    if not async_save:
        torch.save(obj, path)
        return
    t = threading.Thread(target=torch.save, args=(obj, path), daemon=False)
    t.start()
    _ASYNC_THREADS.append(t)


def wait_for_async_saves():
    while _ASYNC_THREADS:
        _ASYNC_THREADS.pop().join()


def _write_latest(save_dir, tag):
    """Atomically point ``latest`` at ``tag`` (tmp file + rename: a crash never leaves a torn tag)."""
    tmp = os.path.join(save_dir, f".latest.{os.getpid()}.tmp")
    with open(tmp, "w") as f:
        f.write(tag)
    os.replace(tmp, os.path.join(save_dir, "latest"))


def _commit_marker(save_dir, tag, rank):
    return os.path.join(save_dir, tag, f".hds_commit_rank{rank}")


def _async_commit(save_dir, tag, rank, world, writers, save_latest, timeout_s=24 * 3600):
    """Background commit of an async save (reference checkpoint engine ``commit(tag)``): every rank marks its tag
    complete once its writer threads joined; rank 0 moves ``latest`` only when all ``world`` markers exist, so a
    rank that dies mid-save leaves ``latest`` on the previous, complete tag. No collectives off the main thread."""
    import time
    for t in writers:
        t.join()
    open(_commit_marker(save_dir, tag, rank), "w").close()
    if rank != 0 or not save_latest:
        return
    t0 = time.time()
    while time.time() - t0 < timeout_s:
        if all(os.path.exists(_commit_marker(save_dir, tag, r)) for r in range(world)):
            _write_latest(save_dir, tag)
            for r in range(world):
                try:
                    os.remove(_commit_marker(save_dir, tag, r))
                except OSError:
                    pass
            return
        time.sleep(0.05)
    logger.warning(f"async checkpoint {tag}: not every rank committed; 'latest' left unchanged")


def _universal_info(engine):
    """``universal_checkpoint_info`` (reference checkpoint/constants.py): how ds_to_universal merges TP slices."""
    from ..checkpoint import constants as C
    info = {C.UNIVERSAL_CHECKPOINT_VERSION_KEY: C.UNIVERSAL_CHECKPOINT_VERSION_VALUE}
    mp = groups.get_model_parallel_world_size() if groups._State.topo is not None else 1
    if mp > 1:
        rep, row, sub = [], [], []
        for n, p in engine.module.named_parameters():
            pat = "^" + re.escape(n) + "$"
            if not getattr(p, "ds_tensor_model_parallel", False):
                rep.append(pat)
            elif getattr(p, "ds_tp_sub_params", None):
                # full (all-TP-ranks) shape: fused rows are the sub-params' full sizes
                shp = tuple(getattr(p, "ds_shape", p.shape))
                sub.append({"patterns": [pat], "shape": (tuple(p.ds_tp_sub_params), ) + shp[1:],
                            "partition_dim": 0})
            elif getattr(p, "ds_tp_cat_dim", 0) == 1:
                row.append(pat)
        info[C.TP_REPLICATED_PARAMETER_PATTERNS] = rep
        info[C.PARAMETER_WITH_ROW_PARALLELISM_PATTERNS] = row
        info[C.PARAMETER_WITH_SUB_PARAMS] = sub
    return info


def _model_state(engine, zopt, stage):
    """Model-state file contents with the reference keys (engine.py:3525-3546)."""
    partitioned = stage == 3 and zopt is not None and zopt.partitioned
    managed = set(zopt.param_to_unit) if zopt is not None else set()
    names = [(n, p) for n, p in engine.module.named_parameters()]
    if partitioned:
        # ZeRO-3: parameters live in the optimizer shards; the module entry keeps buffers + unmanaged params
        module_sd = {n: b.detach().cpu() for n, b in engine.module.named_buffers()}
        module_sd.update({n: p.detach().cpu() for n, p in names if id(p) not in managed})
    else:
        module_sd = _to_cpu(engine.module.state_dict())
    frozen = [(n, p) for n, p in names if not p.requires_grad and id(p) not in managed]
    frozen_shapes = OrderedDict((n, p.shape) for n, p in frozen) if frozen else None
    frozen_frags = None
    if frozen:
        if partitioned:
            W, r = engine.dp_world_size, dist.get_rank(engine.dp_group)
            frozen_frags = {}
            for n, p in frozen:
                flat = p.detach().reshape(-1).float().cpu()
                pn = math.ceil(flat.numel() / W)
                frag = torch.zeros(pn)
                seg = flat[r * pn:(r + 1) * pn]
                frag[:seg.numel()] = seg
                frozen_frags[n] = frag
        else:
            frozen_frags = {n: p.detach().float().cpu() for n, p in frozen}
    shared, seen = {}, {}
    for n, p in engine.module.named_parameters(remove_duplicate=False):
        if id(p) in seen:
            shared[n] = seen[id(p)]
        else:
            seen[id(p)] = n
    if zopt is not None:
        param_shapes = zopt.ref_param_shapes()
    else:
        param_shapes = [OrderedDict((n, p.shape) for n, p in names if p.requires_grad)]
    return dict(
        module=module_sd,
        buffer_names=[n for n, _ in engine.module.named_buffers()],
        optimizer=None,
        param_shapes=param_shapes,
        frozen_param_shapes=frozen_shapes,
        shared_params=shared,
        frozen_param_fragments=frozen_frags,
        lr_scheduler=engine.lr_scheduler.state_dict() if engine.lr_scheduler is not None else None,
        data_sampler=None,
        random_ltd=None,
        sparse_tensor_module_names=[],
        skipped_steps=engine.skipped_steps,
        global_steps=engine.global_steps,
        global_samples=engine.global_samples,
        dp_world_size=engine.dp_world_size,
        mp_world_size=groups.get_model_parallel_world_size() if groups._State.topo is not None else 1,
        ds_config=engine.config,
        ds_version=__version__,
        universal_checkpoint_info=_universal_info(engine),
        hds_module_has_params=not partitioned,
    )


def save_checkpoint(engine, save_dir, tag=None, client_state=None, save_latest=True, exclude_frozen_parameters=False):
    if tag is None:
        tag = f"global_step{engine.global_steps}"
    tag = str(tag)
    async_save = bool(engine._config.checkpoint_config.get("async_save", False))
    wait_for_async_saves()
    rank = dist.get_rank()
    dp_rank = dist.get_rank(engine.dp_group)
    os.makedirs(os.path.join(save_dir, tag), exist_ok=True)
    dist.barrier()
    zopt = engine.optimizer
    stage = engine.zero_optimization_stage()
    state = _model_state(engine, zopt, stage)
    if exclude_frozen_parameters:
        state["frozen_param_shapes"], state["frozen_param_fragments"] = None, None
    state.update(client_state or {})
    n_before = len(_ASYNC_THREADS)
    write_model = (stage == 3 and zopt is not None and zopt.partitioned) or dp_rank == 0
    if write_model:
        _write(state, _ckpt_name(engine, save_dir, tag), async_save)
    if zopt is not None:
        osd_inner = zopt.state_dict()  # collective over the data-parallel groups: every rank participates
        osd = {"optimizer_state_dict": osd_inner, "ds_config": engine.config, "ds_version": __version__}
        if stage > 0 or dp_rank == 0 or (zopt.expert_units and dp_rank < _max_ep(zopt)):
            _write(osd, _optim_name(engine, save_dir, tag), async_save)
    if stage < 3 and zopt is not None and zopt.expert_units and 0 < dp_rank < _max_ep(zopt):
        # other EP ranks' experts (model file of stage 0-2 is written by dp rank 0 only)
        names = {id(p): n for n, p in engine.module.named_parameters()}
        exp = {names[id(p)]: p.detach().cpu() for u in zopt.expert_units for p in u.params}
        _write({"module": exp}, _expert_name(save_dir, tag, dp_rank), async_save)
    if rank == 0:
        try:
            src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoint",
                               "zero_to_fp32.py")
            shutil.copyfile(src, os.path.join(save_dir, "zero_to_fp32.py"))
        except OSError:
            pass
    if async_save:
        writers = _ASYNC_THREADS[n_before:]
        c = threading.Thread(target=_async_commit, args=(save_dir, tag, rank, dist.get_world_size(), writers,
                                                         save_latest), daemon=False)
        c.start()
        _ASYNC_THREADS.append(c)
    else:
        dist.barrier()  # every rank's files are on disk before 'latest' moves
        if rank == 0 and save_latest:
            _write_latest(save_dir, tag)
    log_dist(f"saved checkpoint {save_dir}/{tag}", ranks=[0])
    return True


def _resolve_tag(load_dir, tag):
    if tag is not None:
        return str(tag)
    latest = os.path.join(load_dir, "latest")
    if not os.path.exists(latest):
        logger.warning(f"no 'latest' file in {load_dir}")
        return None
    with open(latest) as f:
        return f.read().strip()


def load_checkpoint(engine, load_dir, tag=None, load_module_strict=True, load_optimizer_states=True,
                    load_lr_scheduler_states=True, load_module_only=False):
    wait_for_async_saves()
    tag = _resolve_tag(load_dir, tag)
    if tag is None:
        return None, None
    zopt = engine.optimizer
    stage = engine.zero_optimization_stage()
    mpath = _ckpt_name(engine, load_dir, tag)
    if not os.path.exists(mpath):
        # model-state file of stage 0-2 lives on dp rank 0 only
        mpath = os.path.join(load_dir, tag, f"mp_rank_{_mp_rank():02d}_model_states.pt")
    from ..checkpoint import compat  # noqa: F401  (reference class names allowed for weights_only loading)
    sd = torch.load(mpath, map_location="cpu", weights_only=True) if os.path.exists(mpath) else {}
    # ZeRO-3 model files hold buffers + unmanaged params only; the weights come from the optimizer shards
    # (universal loads take every weight from zero/<param>/fp32.pt: model-file weights may be TP slices)
    universal = zopt is not None and engine._config.load_universal_checkpoint and not load_module_only
    weightless = stage == 3 or sd.get("hds_module_has_params") is False or universal
    if sd.get("module") is not None:
        msd = sd["module"]
        if weightless:
            managed = set(zopt.param_to_unit) if (zopt is not None and (zopt.partitioned or universal)) else set()
            skip = {n for n, p in engine.module.named_parameters() if id(p) in managed}
            msd = {k: v for k, v in msd.items() if v.numel() > 0 and k not in skip}
        engine.module.load_state_dict(msd, strict=load_module_strict and not weightless)
        if zopt is not None and zopt.expert_units and stage < 3:
            j = dist.get_rank(engine.dp_group) % _max_ep(zopt)
            if j > 0:
                esd = torch.load(_expert_name(load_dir, tag, j), map_location="cpu", weights_only=True)
                engine.module.load_state_dict(esd["module"], strict=False)
        if zopt is not None:
            zopt.refresh_fp32_from_lp()
    if not load_module_only and zopt is not None and engine._config.load_universal_checkpoint:
        from ..checkpoint.universal import load_universal_into
        load_universal_into(zopt, os.path.join(load_dir, tag), load_optimizer_states)
    elif not load_module_only and zopt is not None:
        opath = _optim_name(engine, load_dir, tag)
        if not os.path.exists(opath):
            # stage 0: dp rank 0 (plus one rank per EP position when there are experts) wrote the states
            j = dist.get_rank(engine.dp_group) % _max_ep(zopt) if zopt.expert_units else 0
            prefix = "bf16_" if engine.bfloat16_enabled() else ""
            opath = os.path.join(load_dir, tag, f"{prefix}zero_pp_rank_{j}_mp_rank_{_mp_rank():02d}_optim_states.pt")
        osd = torch.load(opath, map_location="cpu", weights_only=True)
        zopt.load_state_dict(osd["optimizer_state_dict"], load_optimizer_states=load_optimizer_states,
                             param_shapes=sd.get("param_shapes"))
    if not load_module_only:
        if load_lr_scheduler_states and engine.lr_scheduler is not None and sd.get("lr_scheduler") is not None:
            engine.lr_scheduler.load_state_dict(sd["lr_scheduler"])
        engine.global_steps = sd.get("global_steps", 0)
        engine.global_samples = sd.get("global_samples", 0)
        engine.skipped_steps = sd.get("skipped_steps", 0)
        engine.loaded_checkpoint_dp_world_size = sd.get("dp_world_size")
    client = {k: v for k, v in sd.items() if k not in (
        "module", "buffer_names", "optimizer", "param_shapes", "frozen_param_shapes", "shared_params",
        "frozen_param_fragments", "lr_scheduler", "data_sampler", "random_ltd", "sparse_tensor_module_names",
        "skipped_steps", "global_steps", "global_samples", "dp_world_size", "mp_world_size", "ds_config",
        "ds_version", "universal_checkpoint_info", "hds_module_has_params")}
    dist.barrier()
    return os.path.join(load_dir, tag), client


def save_16bit_model(engine, save_dir, save_filename="pytorch_model.bin"):
    """Consolidated 16-bit weights (gathers ZeRO-3 shards); written by rank 0."""
    zopt = engine.optimizer
    if zopt is not None:
        full = zopt.full_fp32_state_dict(engine._param_names)
        sd = {k: v.to(engine.compute_dtype) for k, v in full.items()}
    else:
        sd = _to_cpu(engine.module.state_dict())
    if dist.get_rank() == 0:
        os.makedirs(save_dir, exist_ok=True)
        torch.save(sd, os.path.join(save_dir, save_filename))
    dist.barrier()
    return True
