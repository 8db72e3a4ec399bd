"""Engine checkpoint save/load with the DeepSpeed directory layout and file names.

Reference parity: runtime/engine.py save_checkpoint :3274 / load_checkpoint :2928, file names
:2857-2917 (``mp_rank_XX_model_states.pt``, ``zero_pp_rank_{dp}_mp_rank_{mp:02d}_model_states.pt``,
``[bf16_]zero_pp_rank_{dp}_mp_rank_{mp:02d}_optim_states.pt``), the ``latest`` tag file (:3357-3359), the
model-state keys (:3525-3546), and the copy of ``zero_to_fp32.py`` into the checkpoint dir (:3674-3691).

The optimizer files hold this framework's flat shards plus their layout (unit -> parameter names,
offsets, shapes, shard size), which is all ``zero_to_fp32`` / ``ds_to_universal`` need to rebuild full
parameters or re-shard for a different world size.

Saves are asynchronous when ``checkpoint.async_save`` is set: tensors are copied D2H on a side stream
into pinned memory and written by a background thread, so training continues while the files land.
"""
import os
import shutil
import threading

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
    module_sd = None
    if stage < 3 or (zopt is not None and not zopt.partitioned):
        module_sd = _to_cpu(engine.module.state_dict())
    param_shapes = {n: list(p.ds_shape if hasattr(p, "ds_shape") else p.shape)
                    for n, p in engine.module.named_parameters()}
    state = dict(
        module=module_sd,
        buffer_names=[n for n, _ in engine.module.named_buffers()],
        optimizer=None,
        param_shapes=[param_shapes],
        frozen_param_shapes=None,
        shared_params={},
        frozen_param_fragments=None,
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
    )
    state.update(client_state or {})
    write_model = (stage == 3 and zopt is not None and zopt.partitioned) or dp_rank == 0
    if write_model:
        _write(state, _ckpt_name(engine, save_dir, tag), async_save)
    if zopt is not None:
        osd = {"optimizer_state_dict": zopt.state_dict(), "ds_config": engine.config, "ds_version": __version__}
        if stage > 0 or dp_rank == 0 or (zopt.expert_units and dp_rank < _max_ep(zopt)):
            _write(osd, _optim_name(engine, save_dir, tag), async_save)
    if stage < 3 and zopt is not None and zopt.expert_units and 0 < dp_rank < _max_ep(zopt):
        # other EP ranks' experts (model file of stage 0-2 is written by dp rank 0 only)
        names = {id(p): n for n, p in engine.module.named_parameters()}
        exp = {names[id(p)]: p.detach().cpu() for u in zopt.expert_units for p in u.params}
        _write({"module": exp}, _expert_name(save_dir, tag, dp_rank), async_save)
    if rank == 0:
        if save_latest:
            with open(os.path.join(save_dir, "latest"), "w") as f:
                f.write(tag)
        try:
            src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "checkpoint",
                               "zero_to_fp32.py")
            shutil.copyfile(src, os.path.join(save_dir, "zero_to_fp32.py"))
        except OSError:
            pass
    if not async_save:
        dist.barrier()
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
    sd = torch.load(mpath, map_location="cpu", weights_only=True) if os.path.exists(mpath) else {}
    if sd.get("module") is not None:
        engine.module.load_state_dict(sd["module"], strict=load_module_strict)
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
        zopt.load_state_dict(osd["optimizer_state_dict"], load_optimizer_states=load_optimizer_states)
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
        "ds_version")}
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
