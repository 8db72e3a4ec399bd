"""Checkpoint interoperability with the reference DeepSpeed on-disk schema.

* ``_reference_zero_to_fp32`` re-implements the reference's reconstruction protocol from its documented keys
  (reference utils/zero_to_fp32.py:148-185 parse_optim_states, :252-322 zero-2 merge, :437-487 zero-3 merge);
  it must rebuild the live engine's fp32 weights from OUR files at world 2 and 3 (uneven) for ZeRO-1/2/3.
* ``param_slice_mappings`` must let the reference's ds_to_universal fragment extraction
  (ds_to_universal.py:112-149) rebuild each parameter's fp32 value and moments.
* A universal checkpoint round-trips 2 -> 1 -> 4 ranks with identical fp32 weights and Adam moments.
* A TP=2 checkpoint converts to universal and loads into a TP=1 run.
* Files that carry the reference's pickled helper classes (fragment_address, LossScaler) load with
  ``weights_only=True``.
"""
import glob
import math
import os
import re
import sys
import types
from collections import OrderedDict
from dataclasses import dataclass

import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


def _engine(stage, seed=0, extra=None):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(seed)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": stage}}
    cfg.update(extra or {})
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    return eng


def _train(eng, n, seed):
    g = torch.Generator().manual_seed(seed)
    for _ in range(n):
        x = torch.randint(0, 97, (2, 12), generator=g)
        eng.backward(eng(x, labels=x))
        eng.step()


def _natural(text):
    return [int(c) if c.isdigit() else c for c in re.split(r"(\d+)", text)]


def _reference_zero_to_fp32(ckpt_dir):
    """The reference protocol, written from its documented keys only (no code of this framework)."""
    optim_files = sorted(glob.glob(os.path.join(ckpt_dir, "*_optim_states.pt")), key=_natural)
    sds = [torch.load(f, map_location="cpu", weights_only=True)["optimizer_state_dict"] for f in optim_files]
    stage = sds[0]["zero_stage"]
    world = sds[0]["partition_count"]
    world = max(world) if isinstance(world, list) else world
    assert world == len(optim_files)
    key = "single_partition_of_fp32_groups" if stage <= 2 else "fp32_flat_groups"
    flat_groups = [sd[key] for sd in sds]
    model_file = os.path.join(ckpt_dir, "mp_rank_00_model_states.pt" if stage <= 2 else
                              "zero_pp_rank_0_mp_rank_00_model_states.pt")
    msd = torch.load(model_file, map_location="cpu", weights_only=True)
    param_shapes = msd["param_shapes"]
    out = OrderedDict()
    if stage <= 2:
        for i, shapes in enumerate(param_shapes):
            full = torch.cat([fg[i] for fg in flat_groups])
            off = 0
            for name, shape in shapes.items():
                out[name] = full.narrow(0, off, shape.numel()).view(shape)
                off += shape.numel()
            align = 2 * world
            assert align * math.ceil(off / align) == align * math.ceil(full.numel() / align)
    else:
        merged = {k: v for d in param_shapes for k, v in d.items()}
        per_rank = [torch.cat(list(fg)) for fg in flat_groups]
        off = 0
        for name, shape in merged.items():
            n = shape.numel()
            pn = math.ceil(n / world)
            out[name] = torch.cat([r.narrow(0, off, pn) for r in per_rank]).narrow(0, 0, n).view(shape)
            off += pn
        assert off * world == sum(t.numel() for t in flat_groups[0]) * world
    for alias, owner in msd["shared_params"].items():
        out[alias] = out[owner]
    return out


def _reference_fragments(ckpt_dir, state="fp32"):
    """ds_to_universal.py:112-149 extract_zero_shards + _merge_zero_shards (dp concat), for ZeRO-1/2 files."""
    optim_files = sorted(glob.glob(os.path.join(ckpt_dir, "*_optim_states.pt")), key=_natural)
    frags = {}
    for f in optim_files:
        osd = torch.load(f, map_location="cpu", weights_only=True)["optimizer_state_dict"]
        for g, mapping in enumerate(osd["param_slice_mappings"]):
            flat = (osd["single_partition_of_fp32_groups"][g] if state == "fp32" else
                    osd["base_optimizer_state"]["state"][g][state])
            for name, fa in mapping.items():
                frags.setdefault(name, []).append(flat.narrow(0, fa.start, fa.numel))
    return {k: torch.cat(v) for k, v in frags.items()}


def _write_and_check(rank, world, stage, d):
    eng = _engine(stage)
    _train(eng, 3, 11 + rank)
    eng.save_checkpoint(d, tag="t")
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    from hcache_deepspeed_amd.utils.tensor_fragment import safe_get_full_optimizer_state
    names = dict(eng.module.named_parameters())
    exp_avg = {n: safe_get_full_optimizer_state(p, "exp_avg") for n, p in names.items()}
    torch.distributed.barrier()
    if rank == 0:
        ref = _reference_zero_to_fp32(os.path.join(d, "t"))
        assert set(ref) == set(full)
        for k in full:
            assert torch.equal(ref[k], full[k]), k
        if stage <= 2:
            fr = _reference_fragments(os.path.join(d, "t"))
            ma = _reference_fragments(os.path.join(d, "t"), "exp_avg")
            for k in full:
                assert torch.equal(fr[k], full[k].reshape(-1)), k
                assert torch.allclose(ma[k], exp_avg[k].reshape(-1).float()), k
        # the framework's own consolidation (also copied into the checkpoint dir) agrees
        from hcache_deepspeed_amd.checkpoint.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
        ours = get_fp32_state_dict_from_zero_checkpoint(d, tag="t")
        for k in full:
            assert torch.equal(ours[k], full[k]), k


@pytest.mark.parametrize("stage", [1, 2, 3])
@pytest.mark.parametrize("world", [2, 3])
def test_reference_protocol_reads_our_checkpoint(stage, world, tmp_path):
    run_distributed(_write_and_check, world, stage, str(tmp_path))


# ---------------------------------------------------------------------------------------------
# universal 2 -> 1 -> 4
# ---------------------------------------------------------------------------------------------
def _full_states(eng):
    from hcache_deepspeed_amd.utils.tensor_fragment import (safe_get_full_fp32_param,
                                                            safe_get_full_optimizer_state)
    out = {}
    for n, p in eng.module.named_parameters():
        out[n] = (safe_get_full_fp32_param(p).float().clone(),
                  safe_get_full_optimizer_state(p, "exp_avg").float().clone(),
                  safe_get_full_optimizer_state(p, "exp_avg_sq").float().clone())
    return out


def _u_save(rank, world, stage, d, tag, seed, load_from):
    from hcache_deepspeed_amd.checkpoint import ds_to_universal
    extra = {"checkpoint": {"load_universal": True}} if load_from else None
    eng = _engine(stage, seed=seed, extra=extra)
    if load_from:
        eng.load_checkpoint(d, tag=load_from)
        got = _full_states(eng)
        exp = torch.load(os.path.join(d, "expected.pt"), weights_only=True)
        for k, (w, m, v) in exp.items():
            assert torch.equal(got[k][0], w), ("fp32", k)
            assert torch.equal(got[k][1], m), ("exp_avg", k)
            assert torch.equal(got[k][2], v), ("exp_avg_sq", k)
        assert eng.optimizer.param_groups[0]["step"] == 2
    else:
        _train(eng, 2, 5 + rank)
    if tag:
        eng.save_checkpoint(d, tag=tag)
        states = _full_states(eng)
        if rank == 0:
            torch.save(states, os.path.join(d, "expected.pt"))
            ds_to_universal(d, os.path.join(d, f"{tag}_univ"), tag=tag)
        torch.distributed.barrier()


@pytest.mark.parametrize("stage", [2, 3])
def test_universal_roundtrip_2_1_4(stage, tmp_path):
    d = str(tmp_path)
    run_distributed(_u_save, 2, stage, d, "w2", 0, None)
    run_distributed(_u_save, 1, stage, d, "w1", 77, "w2_univ")
    run_distributed(_u_save, 4, stage, d, None, 99, "w1_univ")


def _universal_layout(rank, world, d):
    """Stage-3 universal files are bare tensors, stage-1/2 files are {'param', 'cat_dim'} dicts (the reference's
    two flavours) and zero/optimizer_state.pt holds the param groups."""
    eng = _engine(3)
    _train(eng, 1, 3)
    eng.save_checkpoint(d, tag="s3")
    from hcache_deepspeed_amd.checkpoint import ds_to_universal
    if rank == 0:
        out = ds_to_universal(d, os.path.join(d, "u3"), tag="s3")
        t = torch.load(os.path.join(out, "zero", "lm_head.weight", "fp32.pt"), weights_only=True)
        assert torch.is_tensor(t) and t.shape == (TINY["vocab_size"], TINY["hidden_size"])
        g = torch.load(os.path.join(out, "zero", "optimizer_state.pt"), weights_only=True)
        assert g["param_groups"][0]["lr"] == pytest.approx(1e-2)
        assert os.path.exists(os.path.join(out, "mp_rank_00_model_states.pt"))


def test_universal_file_flavours(tmp_path):
    run_distributed(_universal_layout, 2, str(tmp_path))


# ---------------------------------------------------------------------------------------------
# tensor parallel: TP=2 checkpoint -> universal -> TP=1
# ---------------------------------------------------------------------------------------------
def _tp_save(rank, world, d):
    eng = _engine(1, extra={"tensor_parallel": {"autotp_size": 2},
                            "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.0}}})
    _train(eng, 2, 5)  # same batch on both TP ranks
    eng.save_checkpoint(d, tag="tp")
    torch.distributed.barrier()
    if rank == 0:
        from hcache_deepspeed_amd.checkpoint import ds_to_universal
        from hcache_deepspeed_amd.checkpoint.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
        ds_to_universal(d, os.path.join(d, "tp_univ"), tag="tp")
        torch.save(get_fp32_state_dict_from_zero_checkpoint(d, tag="tp"), os.path.join(d, "tp_full.pt"))


def _tp_load(rank, world, d):
    eng = _engine(1, seed=5, extra={"checkpoint": {"load_universal": True}})
    eng.load_checkpoint(d, tag="tp_univ")
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    merged = torch.load(os.path.join(d, "tp_full.pt"), weights_only=True)
    assert set(merged) == set(full)
    for k in full:
        assert torch.equal(full[k], merged[k]), k


def _tp_reference_single(d):
    """Single-process training on the same batches: the TP run must have produced these weights."""
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    ref = LlamaForCausalLM(tiny(**TINY))
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    g = torch.Generator().manual_seed(5)
    for _ in range(2):
        x = torch.randint(0, 97, (2, 12), generator=g)
        ref(x, labels=x).backward()
        opt.step()
        opt.zero_grad()
    merged = torch.load(os.path.join(d, "tp_full.pt"), weights_only=True)
    for k, v in ref.state_dict().items():
        assert torch.allclose(merged[k], v, atol=1e-4, rtol=1e-3), k  # Adam amplifies TP reduction-order noise


def test_tp_checkpoint_to_universal_to_tp1(tmp_path):
    d = str(tmp_path)
    run_distributed(_tp_save, 2, d)
    _tp_reference_single(d)
    run_distributed(_tp_load, 1, d)


# ---------------------------------------------------------------------------------------------
# files carrying the reference's pickled classes
# ---------------------------------------------------------------------------------------------
def _save_with_reference_classes(src, dst):
    """Rewrite one of our optimizer files as the reference would pickle it (deepspeed.* class paths)."""
    mods = {}
    for name in ("deepspeed", "deepspeed.utils", "deepspeed.utils.tensor_fragment", "deepspeed.runtime",
                 "deepspeed.runtime.fp16", "deepspeed.runtime.fp16.loss_scaler"):
        mods[name] = types.ModuleType(name)

    @dataclass
    class fragment_address:
        numel: int
        start: int

    class LossScaler:
        pass

    fragment_address.__module__ = "deepspeed.utils.tensor_fragment"
    fragment_address.__qualname__ = "fragment_address"
    LossScaler.__module__ = "deepspeed.runtime.fp16.loss_scaler"
    LossScaler.__qualname__ = "LossScaler"
    mods["deepspeed.utils.tensor_fragment"].fragment_address = fragment_address
    mods["deepspeed.runtime.fp16.loss_scaler"].LossScaler = LossScaler
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    try:
        sd = torch.load(src, weights_only=True)
        osd = sd["optimizer_state_dict"]
        osd["param_slice_mappings"] = [OrderedDict((n, fragment_address(numel=fa.numel, start=fa.start))
                                                   for n, fa in m.items()) for m in osd["param_slice_mappings"]]
        ls = LossScaler()
        ls.cur_scale = 1.0
        ls.dynamic = False
        osd["loss_scaler"] = ls
        osd.pop("hds_param_order")  # a reference file has no such key: the order comes from param_shapes
        torch.save(sd, dst)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def _ref_classes(rank, world, d):
    eng = _engine(2)
    _train(eng, 2, 21)
    eng.save_checkpoint(d, tag="r")
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    torch.distributed.barrier()
    if rank == 0:
        f = glob.glob(os.path.join(d, "r", "*_optim_states.pt"))[0]
        _save_with_reference_classes(f, f)
    torch.distributed.barrier()
    eng2 = _engine(2, seed=3)
    eng2.load_checkpoint(d, tag="r")
    got = eng2.optimizer.full_fp32_state_dict(eng2._param_names)
    for k in full:
        assert torch.equal(got[k], full[k]), k


def test_reference_pickled_classes_load_weights_only(tmp_path):
    run_distributed(_ref_classes, 1, str(tmp_path))


# ---------------------------------------------------------------------------------------------
# async save: 'latest' moves only after every rank committed
# ---------------------------------------------------------------------------------------------
def _async(rank, world, d):
    from hcache_deepspeed_amd.runtime import checkpointing as C
    eng = _engine(2, extra={"checkpoint": {"async_save": True}})
    _train(eng, 1, 1)
    eng.save_checkpoint(d, tag="a1")
    C.wait_for_async_saves()
    torch.distributed.barrier()
    with open(os.path.join(d, "latest")) as f:
        assert f.read() == "a1"
    assert not glob.glob(os.path.join(d, "a1", ".hds_commit_rank*"))
    # rank 1 "dies" before committing tag a2: rank 0's committer must leave 'latest' on a1
    if rank == 0:
        open(C._commit_marker(d, "a2", 0), "w").close() if os.path.isdir(os.path.join(d, "a2")) else None
        os.makedirs(os.path.join(d, "a2"), exist_ok=True)
        C._async_commit(d, "a2", 0, world, [], True, timeout_s=0.5)
        with open(os.path.join(d, "latest")) as f:
            assert f.read() == "a1"
        # once rank 1's marker lands, the commit goes through
        open(C._commit_marker(d, "a2", 1), "w").close()
        C._async_commit(d, "a2", 0, world, [], True, timeout_s=5)
        with open(os.path.join(d, "latest")) as f:
            assert f.read() == "a2"


def test_async_save_commits_latest_after_all_ranks(tmp_path):
    run_distributed(_async, 2, str(tmp_path))


# ---------------------------------------------------------------------------------------------
# reference stage-3 files with several sub-group flats (sub_group_size) and one param group
# ---------------------------------------------------------------------------------------------
def _to_subgroups(ckpt_dir, n_sub):
    """Rewrite our stage-3 files the way the reference's stage 3 writes a model larger than sub_group_size: each
    rank's fp32 / moment flats split into ``n_sub`` sub-group flats, one merged param_shapes group, none of our
    private keys."""
    for f in sorted(glob.glob(os.path.join(ckpt_dir, "*_optim_states.pt")), key=_natural):
        sd = torch.load(f, map_location="cpu", weights_only=True)
        osd = sd["optimizer_state_dict"]
        flat = torch.cat([t.view(-1) for t in osd["fp32_flat_groups"]])
        bounds = [round(i * flat.numel() / n_sub) for i in range(n_sub + 1)]
        cut = lambda t: [t[bounds[i]:bounds[i + 1]].clone() for i in range(n_sub)]  # noqa: E731
        osd["fp32_flat_groups"] = cut(flat)
        st = osd["optimizer_state_dict"]["state"]
        keys = sorted(st)
        moments = {k: cut(torch.cat([st[g][k].view(-1) for g in keys])) for k, v in st[keys[0]].items()
                   if torch.is_tensor(v) and v.dim() == 1}
        osd["optimizer_state_dict"]["state"] = {
            i: {**{k: v for k, v in st[keys[0]].items() if k not in moments}, **{k: moments[k][i] for k in moments}}
            for i in range(n_sub)}
        for k in ("hds_param_order", "hds_group_meta", "hds_optimizer_kind"):
            osd.pop(k, None)
        torch.save(sd, f)
    for f in glob.glob(os.path.join(ckpt_dir, "*_model_states.pt")):
        msd = torch.load(f, map_location="cpu", weights_only=True)
        msd["param_shapes"] = [OrderedDict((n, s) for d in msd["param_shapes"] for n, s in d.items())]
        torch.save(msd, f)


def _subgroup_save(rank, world, d):
    eng = _engine(3)
    _train(eng, 2, 7 + rank)
    eng.save_checkpoint(d, tag="sg")
    states = _full_states(eng)
    torch.distributed.barrier()
    if rank == 0:
        torch.save(states, os.path.join(d, "expected.pt"))
        _to_subgroups(os.path.join(d, "sg"), 3)
    torch.distributed.barrier()


def _subgroup_load(rank, world, d):
    eng = _engine(3, seed=123)
    eng.load_checkpoint(d, tag="sg")
    got = _full_states(eng)
    exp = torch.load(os.path.join(d, "expected.pt"), weights_only=True)
    for k, (w, m, v) in exp.items():
        assert torch.equal(got[k][0], w), ("fp32", k)
        assert torch.equal(got[k][1], m), ("exp_avg", k)
        assert torch.equal(got[k][2], v), ("exp_avg_sq", k)


def test_reference_stage3_subgroup_flats(tmp_path):
    """a reference ZeRO-3 checkpoint of a model over sub_group_size holds more flat groups than param
    groups; zero_to_fp32 and load_checkpoint must walk the merged param_shapes over the concatenated flats."""
    d = str(tmp_path)
    run_distributed(_subgroup_save, 2, d)
    from hcache_deepspeed_amd.checkpoint.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
    ours = get_fp32_state_dict_from_zero_checkpoint(d, tag="sg")
    ref = _reference_zero_to_fp32(os.path.join(d, "sg"))
    exp = torch.load(os.path.join(d, "expected.pt"), weights_only=True)
    for k, (w, _, _) in exp.items():
        assert torch.equal(ours[k], w), k
        assert torch.equal(ref[k], w), k
    run_distributed(_subgroup_load, 2, d)


# ---------------------------------------------------------------------------------------------
# wrapped torch optimizer (lazy state) loading a universal checkpoint before its first step
# ---------------------------------------------------------------------------------------------
def _generic_engine(seed, extra=None):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(seed)
    m = LlamaForCausalLM(tiny(**TINY))
    opt = torch.optim.RMSprop(m.parameters(), lr=1e-3)
    cfg = {"train_micro_batch_size_per_gpu": 2, "zero_optimization": {"stage": 2}}
    cfg.update(extra or {})
    eng, _, _, _ = ds.initialize(model=m, optimizer=opt, config=cfg)
    assert eng.optimizer.kind == "generic"
    return eng


def _generic_flat(eng, key):
    return eng.optimizer._generic_flat_states()[key].clone()


def _generic_save(rank, world, d):
    eng = _generic_engine(0)
    _train(eng, 2, 5)
    eng.save_checkpoint(d, tag="g")
    torch.save({"square_avg": _generic_flat(eng, "square_avg"), "fp32": eng.optimizer.store.master.clone()},
               os.path.join(d, "gexp.pt"))
    from hcache_deepspeed_amd.checkpoint import ds_to_universal
    ds_to_universal(d, os.path.join(d, "g_univ"), tag="g")


def _generic_load(rank, world, d):
    eng = _generic_engine(9, extra={"checkpoint": {"load_universal": True}})
    assert not eng.optimizer._generic_flat_states()  # no state before the first step
    eng.load_checkpoint(d, tag="g_univ")
    exp = torch.load(os.path.join(d, "gexp.pt"), weights_only=True)
    assert torch.equal(eng.optimizer.store.master, exp["fp32"])
    assert torch.equal(_generic_flat(eng, "square_avg"), exp["square_avg"])


def test_universal_moments_load_into_unstepped_generic_optimizer(tmp_path):
    """moments of a wrapped torch optimizer must load from a universal checkpoint even though its
    state does not exist yet (never a silent skip)."""
    d = str(tmp_path)
    run_distributed(_generic_save, 1, d)
    run_distributed(_generic_load, 1, d)


def test_stage3_split_rejects_truncated_flat():
    """A stage-3 sub-group flat shorter than this model's partitions by more than the alignment padding raises
    (it used to load zero-padded weights and moments)."""
    import types
    import pytest
    import torch
    from hcache_deepspeed_amd.runtime.zero.ds_state import _split_like
    groups = [types.SimpleNamespace(part=100, world=2), types.SimpleNamespace(part=50, world=2)]
    out = _split_like(torch.ones(148), groups)  # 2 short: alignment padding, accepted
    assert [t.numel() for t in out] == [100, 50] and float(out[1][-1]) == 0.0
    with pytest.raises(ValueError):
        _split_like(torch.ones(120), groups)
