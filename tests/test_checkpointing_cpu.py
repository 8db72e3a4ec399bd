"""Activation checkpointing replays the model-parallel RNG tracker (reference checkpointing.py:539,645-660)."""
import pytest
import torch

import hcache_deepspeed_amd.runtime.activation_checkpointing.checkpointing as ck


@pytest.fixture
def tracker():
    t = ck.get_cuda_rng_tracker()
    saved = t.get_states(), set(t.seeds_)
    t.reset()
    t.add("model-parallel-rng", 1234)
    yield t
    t.states_, t.seeds_ = saved


def _block(x, w):
    # dropout inside a model-parallel region draws from the tracker, dropout outside from the default generator
    y = x @ w
    with ck.get_cuda_rng_tracker().fork():
        y = torch.nn.functional.dropout(y, 0.5, training=True)
    return torch.nn.functional.dropout(y.tanh(), 0.3, training=True) @ w


@pytest.mark.parametrize("kind", ["non_reentrant", "saved_inputs"])
def test_recompute_replays_tracker_dropout(tracker, kind):
    torch.manual_seed(0)
    w = torch.randn(16, 16, requires_grad=True)
    x = torch.randn(8, 16, requires_grad=True)
    st = tracker.get_states()
    torch.manual_seed(5)
    ref = _block(x, w)
    ref.square().sum().backward()
    gw, gx = w.grad.clone(), x.grad.clone()
    after_ref = tracker.get_states()["model-parallel-rng"].clone()
    w.grad = x.grad = None
    tracker.set_states(dict(st))
    torch.manual_seed(5)
    if kind == "non_reentrant":
        out = ck.checkpoint(_block, x, w)
    else:
        out = ck.checkpoint_saved_inputs(_block, x, w)
    # the tracker advances between forward and backward (another region drew from it): the recompute must still use
    # the forward's state
    with tracker.fork():
        torch.rand(100)
    advanced = tracker.get_states()["model-parallel-rng"].clone()
    out.square().sum().backward()
    torch.testing.assert_close(out, ref)
    torch.testing.assert_close(w.grad, gw)
    torch.testing.assert_close(x.grad, gx)
    # the recompute left the backward-time tracker state alone
    assert torch.equal(tracker.get_states()["model-parallel-rng"], advanced)
    assert not torch.equal(advanced, after_ref)
