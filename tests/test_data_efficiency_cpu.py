"""Curriculum learning, data sampler, random-LTD, progressive layer drop, eigenvalue, MoQ (reference
tests/unit/runtime/test_data_efficiency.py, test_pld.py, test_ds_config... strategies)."""
import os

import numpy as np
import pytest
import torch


def test_curriculum_schedules():
    from hcache_deepspeed_amd.runtime.data_pipeline import CurriculumScheduler
    lin = CurriculumScheduler({"min_difficulty": 8, "max_difficulty": 64, "schedule_type": "fixed_linear",
                               "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 8}})
    vals = [lin.update_difficulty(s) for s in range(0, 13)]
    assert vals[0] == 8 and vals[-1] == 64 and all(a <= b for a, b in zip(vals, vals[1:]))
    assert all(v % 8 == 0 for v in vals)
    root = CurriculumScheduler({"min_difficulty": 8, "max_difficulty": 64, "schedule_type": "fixed_root",
                                "schedule_config": {"total_curriculum_step": 10, "difficulty_step": 8,
                                                    "root_degree": 2}})
    assert root.get_difficulty(3) >= lin.get_difficulty(3)
    disc = CurriculumScheduler({"min_difficulty": 1, "max_difficulty": 3, "schedule_type": "fixed_discrete",
                                "schedule_config": {"difficulty": [1, 2, 3], "max_step": [5, 10]}})
    assert [disc.get_difficulty(s) for s in (1, 5, 6, 10, 11)] == [1, 1, 2, 2, 3]


def test_data_sampler_respects_difficulty():
    from hcache_deepspeed_amd.runtime.data_pipeline import DeepSpeedDataSampler
    metric = np.arange(1000) % 100  # difficulty 0..99
    s = DeepSpeedDataSampler(metric, 32, 8, 0, 2, {"min_difficulty": 10, "max_difficulty": 100,
                                                   "schedule_type": "fixed_linear",
                                                   "schedule_config": {"total_curriculum_step": 5,
                                                                       "difficulty_step": 10}})
    it = iter(s)
    first = [next(it) for _ in range(2)]  # rank 0's two micro-batches of step 1
    assert all(metric[i] <= 28 for mb in first for i in mb)
    sd = s.state_dict()
    s2 = DeepSpeedDataSampler(metric, 32, 8, 0, 2)
    s2.load_state_dict(sd)
    assert s2.consumed_samples == 32


def test_random_ltd_gather_scatter_and_layer():
    from hcache_deepspeed_amd.runtime.data_pipeline import (RandomLayerTokenDrop, RandomLTDScheduler, gpt_sample_tokens,
                                                            token_gather, token_scatter)
    x = torch.randn(2, 16, 8)
    idx = gpt_sample_tokens(6, 16, 2)[0]
    assert (idx[:, 1:] > idx[:, :-1]).all()
    part = token_gather(x, idx)
    assert torch.equal(part[1, 3], x[1, idx[1, 3]])
    y = token_scatter(x, part * 2, idx)
    mask = torch.zeros(2, 16, dtype=torch.bool)
    mask[torch.arange(2)[:, None], idx] = True
    assert torch.allclose(y[mask], x[mask] * 2) and torch.equal(y[~mask], x[~mask])
    sch = RandomLTDScheduler({"min_value": 4, "max_value": 16, "schedule_config": {"require_steps": 10,
                                                                                  "seq_per_step": 4}})
    layer = RandomLayerTokenDrop(torch.nn.Linear(8, 8), sch)
    layer.train()
    out = layer(x)
    assert out.shape == x.shape and (out == x).all(-1).sum() >= 2 * (16 - 4)
    assert sch.update_seq(10) == 16


def test_pld_and_engine_curriculum():
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.runtime.progressive_layer_drop import ProgressiveLayerDrop
    p = ProgressiveLayerDrop(theta=0.5, gamma=0.1)
    p.update_state(10)
    assert 0.5 < p.get_theta() < 1.0
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29641"))
    seen = []

    class M(torch.nn.Module):

        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(4, 4)

        def forward(self, x, labels=None, progressive_layer_drop=False, pld_theta=1.0):
            seen.append((x.shape[1], pld_theta))
            return self.lin(x.float()).sum()

    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           "curriculum_learning": {"enabled": True, "curriculum_type": "seqlen", "min_difficulty": 2,
                                   "max_difficulty": 8, "schedule_type": "fixed_linear",
                                   "schedule_config": {"total_curriculum_step": 3, "difficulty_step": 2}},
           "progressive_layer_drop": {"enabled": True, "theta": 0.5, "gamma": 0.5}}
    eng, _, _, _ = ds.initialize(model=M(), config=cfg)
    for _ in range(4):
        x = torch.randn(2, 8, 4)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
    lens = [s for s, _ in seen]
    assert lens[0] < 8 and lens[-1] == 8 and lens == sorted(lens)
    assert seen[0][1] == 1.0 and seen[-1][1] < 1.0


def test_eigenvalue_quadratic():
    from hcache_deepspeed_amd.runtime.eigenvalue import Eigenvalue
    torch.manual_seed(0)
    lin = torch.nn.Linear(4, 1, bias=False)
    A = torch.diag(torch.tensor([5.0, 1.0, 0.5, 0.1]))
    w = lin.weight
    loss = 0.5 * (w @ A @ w.t()).sum()
    ev = Eigenvalue(max_iter=200, tol=1e-6)
    res = ev.compute_eigenvalue(torch.nn.ModuleList([lin]), loss=loss)
    assert res[0][0] == pytest.approx(1.0)  # normalised by the max
    ev2 = Eigenvalue(max_iter=200, tol=1e-6)
    ev2.post_process = lambda d: d
    raw = ev2.compute_eigenvalue(torch.nn.ModuleList([lin]), loss=0.5 * (w @ A @ w.t()).sum())
    assert raw[0][0] == pytest.approx(5.0, rel=1e-3)


def test_moq_quantizer_schedule():
    from hcache_deepspeed_amd.runtime.quantize import Quantizer
    p = torch.nn.Parameter(torch.randn(16, 16))
    p.start_bits, p.target_bits, p.q_period = 8, 4, 2
    q = Quantizer(q_groups=4)
    orig = p.data.clone()
    for _ in range(6):
        q.quantize([[p]], overflow=False)
    assert p.start_bits == 4 or p.start_bits < 8
    assert p.data.unique().numel() <= 4 * 2**8
    assert (p.data - orig).abs().max() < orig.abs().max()
