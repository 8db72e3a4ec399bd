"""Fault injection + checkpoint resume (SURVEY.md §5.3 plan: kill rank k at step n, restart, resume from the
latest checkpoint and continue exactly as an uninterrupted run), ZeRO safe_mode layout check, debug-sync mode."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_checkpoint_cpu import _engine


def _steps(eng, start, n, rank, save_dir=None):
    losses = []
    for s in range(start, start + n):
        g = torch.Generator().manual_seed(1000 * s + rank)  # data depends only on (step, rank): resumable
        x = torch.randint(0, 97, (2, 12), generator=g)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
        if save_dir is not None:
            eng.save_checkpoint(save_dir)
    return losses


def _faulty_run(rank, world, d):
    os.environ["HDS_FAULT_INJECT"] = "1:3:raise"
    eng = _engine(3)
    _steps(eng, 0, 5, rank, save_dir=d)  # rank 1 raises inside step 3, before saving it


def _resumed_run(rank, world, d, ref_path):
    os.environ.pop("HDS_FAULT_INJECT", None)
    eng = _engine(3, seed=77)
    eng.load_checkpoint(d)
    assert eng.global_steps == 2  # the last checkpoint completed before the fault
    tail = _steps(eng, eng.global_steps, 3, rank)
    ref = torch.load(ref_path, weights_only=True)[rank]
    assert tail == pytest.approx(ref[2:], rel=1e-5, abs=1e-5)


def _reference_run(rank, world, out):
    eng = _engine(3)
    losses = _steps(eng, 0, 5, rank)
    allv = [None] * world
    torch.distributed.all_gather_object(allv, losses)
    if rank == 0:
        torch.save(allv, out)


def test_fault_then_resume(tmp_path):
    ref = str(tmp_path / "ref.pt")
    run_distributed(_reference_run, 2, ref)
    d = str(tmp_path / "ckpt")
    with pytest.raises(AssertionError, match="injected fault"):
        run_distributed(_faulty_run, 2, d, timeout=120)
    with open(os.path.join(d, "latest")) as f:
        assert f.read().strip() == "global_step2"
    run_distributed(_resumed_run, 2, d, ref)


def test_fault_spec_parsing():
    from hcache_deepspeed_amd.utils.fault_injection import FaultInjector, InjectedFault
    os.environ["HDS_FAULT_INJECT"] = "0:2,3:5:exit"
    try:
        fi = FaultInjector({"rank": 1, "step": 9, "mode": "raise"})
    finally:
        del os.environ["HDS_FAULT_INJECT"]
    assert fi.specs == [(0, 2, "raise"), (3, 5, "exit"), (1, 9, "raise")]
    fi.maybe_fire(0, 1)
    with pytest.raises(InjectedFault):
        fi.maybe_fire(0, 2)
    assert not fi.enabled  # fires once
    with pytest.raises(ValueError):
        FaultInjector({"rank": 0, "step": 1, "mode": "explode"})


def _safe_mode_mismatch(rank, world):
    from hcache_deepspeed_amd.runtime.utils import assert_ints_same_as_other_ranks
    assert_ints_same_as_other_ranks([1, 2, 3])
    with pytest.raises(RuntimeError, match="disagree"):
        assert_ints_same_as_other_ranks([1, 2, 3 + rank], what="unit sizes")
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from tests.test_zero_cpu import TINY
    m = LlamaForCausalLM(tiny(**TINY))
    ds.initialize(model=m, config={"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW"},
                                   "zero_optimization": {"stage": 3, "safe_mode": True}})


def test_safe_mode():
    run_distributed(_safe_mode_mismatch, 2)
