"""Per-tensor activation plan (offload/act_plan.py) on CPU: keep / spill / recompute per tensor class must give
the same gradients as a plain run, recipes must resolve for the classes that have them, and the planner must pick
the cheapest way to free the over-budget bytes."""
import pytest
import torch

from hcache_deepspeed_amd.models import llama
from hcache_deepspeed_amd.offload import act_plan
from hcache_deepspeed_amd.offload.act_plan import KEEP, RECOMPUTE, SPILL, PlannedActivationCache, plan_tensors
from hcache_deepspeed_amd.runtime.zero.linear import wrap_memory_efficient_linears


def _model(seed=0):
    torch.manual_seed(seed)
    m = llama.build("tiny", num_hidden_layers=3, vocab_size=128, hidden_size=64, intermediate_size=96,
                    num_attention_heads=4, num_key_value_heads=2, head_dim=16)
    wrap_memory_efficient_linears(m)
    return m


def _grads(model, ids, cache=None):
    model.zero_grad(set_to_none=True)
    if cache is not None:
        with cache.forward_context():
            loss = model(ids, labels=ids)
    else:
        loss = model(ids, labels=ids)
    loss.backward()
    return loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}


CLASSES = ["resid#0", "norm_out#0", "qkv#0", "attn_out#0", "attn_lse#0", "resid#1", "norm_out#1", "linear_out#0",
           "glu_out#0"]


@pytest.mark.parametrize("mode", ["recompute_all", "spill_all", "mixed", "recompute_chain"])
def test_plan_matches_plain_backward(mode):
    model = _model()
    ids = torch.randint(0, 128, (2, 16))
    ref_loss, ref = _grads(model, ids)
    if mode == "recompute_all":
        forced = {c: RECOMPUTE for c in CLASSES}
    elif mode == "spill_all":
        forced = {c: SPILL for c in CLASSES}
    elif mode == "mixed":
        forced = {"resid#0": SPILL, "norm_out#0": RECOMPUTE, "qkv#0": RECOMPUTE, "attn_out#0": SPILL,
                  "resid#1": RECOMPUTE, "norm_out#1": RECOMPUTE, "linear_out#0": SPILL, "glu_out#0": RECOMPUTE}
    else:  # a recomputed tensor whose source is itself recomputed (x2 <- h2 <- o W_o + h1)
        forced = {"resid#1": RECOMPUTE, "norm_out#1": RECOMPUTE, "linear_out#0": RECOMPUTE, "glu_out#0": RECOMPUTE}
    cache = PlannedActivationCache(torch.device("cpu"), forced=forced, min_bytes=0, min_layers_resident=0)
    cache.attach(model)
    for _ in range(2):
        loss, g = _grads(model, ids, cache)
        assert torch.equal(loss, ref_loss)
        assert g.keys() == ref.keys()
        for n in ref:
            torch.testing.assert_close(g[n], ref[n], rtol=0, atol=0, msg=n)
    assert act_plan._ACTIVE is None
    if mode != "spill_all":
        assert cache._rec_acc > 0  # recipes resolved and were planned
    else:
        assert cache.bytes_offloaded > 0


def test_recipes_resolve_for_expected_classes():
    model = _model()
    ids = torch.randint(0, 128, (2, 16))
    cache = PlannedActivationCache(torch.device("cpu"), forced={c: RECOMPUTE for c in CLASSES}, min_bytes=0,
                                   min_layers_resident=0)
    cache.attach(model)
    seen = {}
    orig = cache._pack

    def spy(t):
        r = orig(t)
        if isinstance(r, act_plan._Ref):
            seen.setdefault(r.h.cls, set()).add(r.h.action)
        return r

    cache._pack = spy
    with cache.forward_context():
        loss = model(ids, labels=ids)
    loss.backward()
    # recomputable: norm outputs, h2 (o W_o + h1, the O projection inlined), the gate|up output, the GLU output,
    # qkv (projection + RoPE); not: the block input h1, attention output and LSE
    for c in ("norm_out#0", "norm_out#1", "resid#1", "linear_out#0", "glu_out#0", "qkv#0"):
        assert seen[c] == {RECOMPUTE}, (c, seen.get(c))
    for c in ("attn_out#0", "attn_lse#0"):
        assert seen[c] == {KEEP}, (c, seen.get(c))


def test_shared_saves_use_one_handle():
    """The attention output is saved by attention and (as a view) by the O projection: one handle, spilled once."""
    model = _model()
    ids = torch.randint(0, 128, (1, 16))
    cache = PlannedActivationCache(torch.device("cpu"), forced={"attn_out#0": SPILL}, min_bytes=0,
                                   min_layers_resident=0)
    cache.attach(model)
    with cache.forward_context():
        loss = model(ids, labels=ids)
    per_layer = {l: len(v) for l, v in cache.by_layer.items()}
    assert per_layer == {0: 1, 1: 1, 2: 1}
    h = cache.by_layer[0][0]
    assert h.refs == 2
    loss.backward()
    assert h.host is None and h.dev is None  # released after its two consumers


def test_planner_prefers_cheap_recompute_then_spill_then_gemm_recompute():
    GB = 10**9
    items = {}
    for l in range(4):
        items[(l, "norm")] = 1 * GB   # 0.5 ms/GB
        items[(l, "gemm")] = 2 * GB   # 2.5 ms/GB
        items[(l, "attn")] = 1 * GB   # not recomputable
    rec = {"norm": 0.5, "gemm": 5.0}
    base = 100 * GB
    budget = base + sum(items.values()) + (1 << 30)
    acts, cost = plan_tensors(items, base, budget, rec, spill_cap_bytes=0)
    assert all(a == KEEP for a in acts.values()) and cost == 0.0
    # 3 GB over: the cheap recompute class covers it
    acts, cost = plan_tensors(items, base, budget - 3 * GB, rec, spill_cap_bytes=0)
    assert sum(1 for k, a in acts.items() if a == RECOMPUTE and k[1] == "norm") == 3
    assert all(a != SPILL for a in acts.values())
    # 9 GB over: all 4 norm items (4 GB), then spills within the 3 GB cap, earliest block and the
    # non-recomputable class first, then GEMM recomputes
    acts, cost = plan_tensors(items, base, budget - 9 * GB, rec, spill_cap_bytes=3 * GB, no_spill_layers=[3])
    assert all(acts[(l, "norm")] == RECOMPUTE for l in range(4))
    spilled = sorted(k for k, a in acts.items() if a == SPILL)
    assert spilled[0] == (0, "attn") and all(k[0] != 3 for k in spilled)
    assert sum(items[k] for k in spilled) <= 3 * GB
    freed = sum(items[k] for k, a in acts.items() if a != KEEP)
    assert freed >= 9 * GB


def test_calibration_step_times_recipes_without_consuming():
    """The calibration step (everything spilled) runs each class's recipe once to time it; that peek must not
    consume any handle (an inlined recipe's sources included) -- gradients stay exact."""
    model = _model()
    ids = torch.randint(0, 128, (2, 16))
    ref_loss, ref = _grads(model, ids)
    cache = PlannedActivationCache(torch.device("cpu"), min_bytes=0, min_layers_resident=1)
    cache.attach(model)
    cache._stage = 1  # what forward_context's planner does on the GPU before the calibration forward
    loss, g = _grads(model, ids, cache)
    assert torch.equal(loss, ref_loss)
    for n in ref:
        torch.testing.assert_close(g[n], ref[n], rtol=0, atol=0, msg=n)
    assert {"norm_out#0", "resid#1", "linear_out#0", "glu_out#0", "qkv#0"} <= set(cache.rec_ms), cache.rec_ms
    assert cache._cal_items and cache.bytes_offloaded > 0


def test_closed_loop_backs_off_capacity_not_price():
    """A spilling step whose forward slowed by more than twice the modelled cost shrinks the spill capacity by a
    quarter (floor 1/4) and keeps the per-GB price; a no-spill forward refines the base forward time."""

    class _Ev:
        def __init__(self, ms):
            self.ms = ms

        def synchronize(self):
            pass

        def elapsed_time(self, other):
            return other.ms - self.ms

    c = PlannedActivationCache(torch.device("cpu"), spill_cost_ms_per_gb=0.6)
    c._stage, c.t_fwd_ms, c.pcie_gbps = 3, 700.0, 56.0
    c.items, c._peak_all, c.budget, c.actions = {}, 0, 1 << 40, {}
    cap0 = c.spill_capacity()
    for slow_ms, scale in ((60.0, 0.75), (5.0, 0.75), (90.0, 0.5625)):
        c.step_spill_bytes = 29 * 10**9
        c._fwd_ev = (_Ev(0.0), _Ev(700.0 + slow_ms))
        c._turn_peak = None
        c._advance_plan()
        assert c.cap_scale == pytest.approx(scale)
        assert c.spill_cost == 0.6
    assert c.spill_capacity() == pytest.approx(0.5625 * cap0, rel=1e-6)
    for _ in range(10):
        c.step_spill_bytes = 29 * 10**9
        c._fwd_ev = (_Ev(0.0), _Ev(900.0))
        c._advance_plan()
    assert c.cap_scale == 0.25
    c.step_spill_bytes = 0
    c._fwd_ev = (_Ev(0.0), _Ev(650.0))
    c._advance_plan()
    assert c.t_fwd_ms == 650.0
