"""Standalone FP16_Optimizer / FP16_UnfusedOptimizer / BF16_Optimizer vs plain fp32 training, overflow skipping and
dynamic loss-scale updates, state_dict round trip.

Reference test analogue: tests/unit/runtime/half_precision/test_fp16.py / test_bf16.py and
test_dynamic_loss_scale.py (overflow skips the step and halves the scale; steady steps grow it after the window).
"""
import pytest
import torch

from hcache_deepspeed_amd.runtime.bf16_optimizer import BF16_Optimizer
from hcache_deepspeed_amd.runtime.fp16.fused_optimizer import FP16_Optimizer, FP16_UnfusedOptimizer


def _model(dtype):
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4)).to(dtype)


@pytest.mark.parametrize("cls,dtype", [(FP16_Optimizer, torch.float16), (FP16_UnfusedOptimizer, torch.float16),
                                       (BF16_Optimizer, torch.bfloat16)])
def test_wrapper_tracks_fp32_training(cls, dtype):
    ref = _model(torch.float32)
    m = _model(dtype)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    kw = {"static_loss_scale": 128.0} if cls is not BF16_Optimizer else {}
    opt = cls(torch.optim.SGD(m.parameters(), lr=0.1), **kw)
    x, y = torch.randn(32, 8), torch.randn(32, 4)
    for _ in range(5):
        ropt.zero_grad()
        torch.nn.functional.mse_loss(ref(x), y).backward()
        ropt.step()
        opt.zero_grad()
        opt.backward(torch.nn.functional.mse_loss(m(x.to(dtype)).float(), y))
        assert opt.step() is True
    for p, q in zip(ref.parameters(), m.parameters()):
        assert torch.allclose(p, q.float(), atol=2e-2), (p - q.float()).abs().max()
    # fp32 masters hold the full-precision trajectory
    master = opt.fp32_groups[0][0]
    assert master.dtype == torch.float32


def test_dynamic_loss_scale_overflow_skip_and_state_roundtrip():
    m = _model(torch.float16)
    opt = FP16_Optimizer(torch.optim.SGD(m.parameters(), lr=0.1), dynamic_loss_scale=True,
                         dynamic_loss_args={"init_scale": 2.0**10, "scale_window": 2, "delayed_shift": 1})
    before = [p.detach().clone() for p in m.parameters()]
    opt.zero_grad()
    for p in m.parameters():
        p.grad = torch.full_like(p, float("inf"))
    assert opt.step() is False and opt.overflow
    assert opt.cur_scale == 2.0**9
    assert all(torch.equal(a, b) for a, b in zip(before, m.parameters()))
    x = torch.randn(4, 8).half()
    for _ in range(2):
        opt.zero_grad()
        opt.backward(m(x).float().pow(2).mean())
        assert opt.step()
    assert opt.cur_scale == 2.0**10  # grew back after scale_window clean steps
    sd = opt.state_dict()
    m2 = _model(torch.float16)
    opt2 = FP16_Optimizer(torch.optim.SGD(m2.parameters(), lr=0.1), dynamic_loss_scale=True)
    opt2.load_state_dict(sd)
    assert opt2.cur_scale == opt.cur_scale
    assert all(torch.equal(a, b) for a, b in zip(m.parameters(), m2.parameters()))
