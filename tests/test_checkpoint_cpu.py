"""Checkpoint save/load round trips (reference tests/unit/checkpoint/common.py checkpoint_correctness_verification):
train -> save -> fresh engine -> load -> identical weights/optimizer state and identical continued training;
zero_to_fp32 consolidation; universal checkpoint re-sharding from 2 ranks to 1."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


def _engine(stage, seed=0):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(seed)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "scheduler": {"type": "WarmupLR", "params": {"warmup_num_steps": 5, "warmup_max_lr": 1e-2}},
           "zero_optimization": {"stage": stage}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    return eng


def _train(eng, n, seed):
    g = torch.Generator().manual_seed(seed)
    losses = []
    for _ in range(n):
        x = torch.randint(0, 97, (2, 12), generator=g)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    return losses


def _roundtrip(rank, world, stage, d):
    eng = _engine(stage)
    _train(eng, 3, 1 + rank)
    eng.save_checkpoint(d, client_state={"my_key": 7})
    cont = _train(eng, 2, 100 + rank)
    full_a = eng.optimizer.full_fp32_state_dict(eng._param_names)
    eng2 = _engine(stage, seed=123)  # different init, must be overwritten by load
    path, client = eng2.load_checkpoint(d)
    assert client["my_key"] == 7
    assert eng2.global_steps == 3
    cont2 = _train(eng2, 2, 100 + rank)
    full_b = eng2.optimizer.full_fp32_state_dict(eng2._param_names)
    assert cont == pytest.approx(cont2, rel=1e-5, abs=1e-5)
    for k in full_a:
        assert torch.allclose(full_a[k], full_b[k], atol=1e-6), k
    # zero_to_fp32 consolidation equals the live engine's weights at the save point
    if rank == 0:
        from hcache_deepspeed_amd.checkpoint.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
        assert os.path.exists(os.path.join(d, "zero_to_fp32.py"))
        sd = get_fp32_state_dict_from_zero_checkpoint(d)
        assert set(sd.keys()) == set(full_a.keys())


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_checkpoint_roundtrip_world2(stage, tmp_path):
    run_distributed(_roundtrip, 2, stage, str(tmp_path))


def _save_w2(rank, world, d):
    eng = _engine(3)
    _train(eng, 2, 5 + rank)
    eng.save_checkpoint(d, tag="t2")
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)  # collective: every rank
    if rank == 0:
        torch.save(full, os.path.join(d, "expected.pt"))


def _load_w1_universal(rank, world, d):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.checkpoint import ds_to_universal
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    ds_to_universal(d, os.path.join(d, "univ"), tag="t2")
    torch.manual_seed(9)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": 3}, "checkpoint": {"load_universal": True}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    from hcache_deepspeed_amd.checkpoint.universal import load_universal_into
    load_universal_into(eng.optimizer, os.path.join(d, "univ"))
    got = eng.optimizer.full_fp32_state_dict(eng._param_names)
    exp = torch.load(os.path.join(d, "expected.pt"), weights_only=True)
    for k in exp:
        assert torch.allclose(got[k], exp[k]), k
    _train(eng, 1, 3)


def test_universal_reshard_2_to_1(tmp_path):
    run_distributed(_save_w2, 2, str(tmp_path))
    run_distributed(_load_w1_universal, 1, str(tmp_path))


def _save_w2_stage(rank, world, d, stage):
    eng = _engine(stage)
    _train(eng, 2, 5 + rank)
    eng.save_checkpoint(d, tag="t")


@pytest.mark.parametrize("stage", [1, 3])
def test_ds_to_universal_workers_strict_inject(stage, tmp_path):
    """Parallel extraction / merge give byte-identical files to the serial conversion; keep_temp_folder keeps the
    slices; a ZeRO-1/2 source without universal_checkpoint_info needs inject_missing_state; strict fails on a
    parameter that did not convert."""
    from hcache_deepspeed_amd.checkpoint.ds_to_universal import main, parse_arguments
    from hcache_deepspeed_amd.checkpoint.universal import ds_to_universal
    d = str(tmp_path)
    run_distributed(_save_w2_stage, 2, d, stage)
    a, b = os.path.join(d, "ua"), os.path.join(d, "ub")
    ds_to_universal(d, a, tag="t")
    main(parse_arguments(["--input_folder", d, "--output_folder", b, "--tag", "t", "--num_extract_workers", "3",
                          "--num_merge_workers", "2", "--keep_temp_folder"]))
    assert os.path.isdir(os.path.join(b, "tmp")) and not os.path.isdir(os.path.join(a, "tmp"))
    with open(os.path.join(d, "latest_universal")) as f:
        assert f.read().strip() == "ub"
    names = sorted(os.listdir(os.path.join(a, "zero")))
    assert names == sorted(os.listdir(os.path.join(b, "zero"))) and len(names) > 3
    for n in names:
        pa = os.path.join(a, "zero", n)
        if not os.path.isdir(pa):
            continue
        for f in os.listdir(pa):
            x = torch.load(os.path.join(pa, f), weights_only=True)
            y = torch.load(os.path.join(b, "zero", n, f), weights_only=True)
            x, y = (v["param"] if isinstance(v, dict) else v for v in (x, y))
            assert torch.equal(x, y) if torch.is_tensor(x) else x == y, (n, f)  # step.pt holds an int
    # a source missing universal_checkpoint_info
    mf = [f for f in os.listdir(os.path.join(d, "t")) if f.endswith("model_states.pt")]
    for f in mf:
        p = os.path.join(d, "t", f)
        sd = torch.load(p, weights_only=False)
        sd.pop("universal_checkpoint_info", None)
        torch.save(sd, p)
    if stage <= 2:
        with pytest.raises(ValueError, match="universal_checkpoint_info"):
            ds_to_universal(d, os.path.join(d, "uc"), tag="t")
    out = ds_to_universal(d, os.path.join(d, "uc"), tag="t", inject_missing_state=True)
    sd = torch.load(os.path.join(out, "mp_rank_00_model_states.pt"), weights_only=False)
    assert stage == 3 or sd["universal_checkpoint_info"]["universal_checkpoint_version"] == 0.2
    # strict: a converted parameter that disagrees with the model states' weights fails the conversion
    bad = None
    for f in mf:
        p = os.path.join(d, "t", f)
        sd = torch.load(p, weights_only=False)
        bad = bad or next((k for k, v in sd["module"].items() if torch.is_tensor(v) and v.numel() > 4), None)
        if bad is None:
            return  # stage 3: the model states hold no full weights to check against
        sd["module"][bad] = torch.zeros(3)
        torch.save(sd, p)
    with pytest.raises(ValueError, match="model states"):
        ds_to_universal(d, os.path.join(d, "ud"), tag="t", inject_missing_state=True)
    ds_to_universal(d, os.path.join(d, "ud"), tag="t", inject_missing_state=True, strict=False)
