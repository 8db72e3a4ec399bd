"""Mixture of Experts: routing/dispatch/combine numerics, expert parallelism (all-to-all) on gloo, and
ZeRO 0-3 with expert-data-parallel sharding (reference tests/unit/moe/test_moe.py strategy: MoE layer
inside ZeRO stages, EP sizes dividing the world, outputs matched against a non-EP computation)."""
import pytest
import torch
import torch.nn.functional as F

from tests.dist_utils import run_distributed


def _dense_moe_ref(x, wg, w13, w2, k):
    """Explicit per-token sum_j w_j * expert_{e_j}(x) (no capacity limit)."""
    probs = torch.softmax(x.float() @ wg.float().t(), -1)
    topw, topi = torch.topk(probs, k, -1)
    topw = topw / topw.sum(-1, keepdim=True)
    out = torch.zeros_like(x)
    for t in range(x.shape[0]):
        for j in range(k):
            e = int(topi[t, j])
            h = w13[e] @ x[t]
            I = h.shape[0] // 2
            y = w2[e] @ (F.silu(h[:I]) * h[I:])
            out[t] = out[t] + topw[t, j] * y
    return out


def test_topk_route_positions_and_capacity():
    from hcache_deepspeed_amd.ops.moe import topk_route
    torch.manual_seed(0)
    logits = torch.randn(10, 4)
    expert, pos, w, C, l_aux, counts = topk_route(logits, 2, capacity_factor=1.0, min_capacity=1)
    assert expert.shape == (10, 2) and pos.shape == (10, 2)
    assert C == 5  # ceil(10 * 2 / 4 * 1.0)
    # k-major priority: positions are a dense 0..n-1 ranking inside each expert
    for e in range(4):
        ps = sorted(int(p) for p, ee in zip(pos.reshape(-1), expert.reshape(-1)) if ee == e)
        assert ps == list(range(len(ps)))
        assert int(counts[e]) == len(ps)
    # every first choice ranks before any second choice of the same expert
    for e in range(4):
        first = [int(pos[t, 0]) for t in range(10) if expert[t, 0] == e]
        second = [int(pos[t, 1]) for t in range(10) if expert[t, 1] == e]
        if first and second:
            assert max(first) < min(second)
    assert torch.allclose(w.sum(-1), torch.ones(10))
    assert float(l_aux) > 0


def test_moe_layer_matches_dense_reference_and_grads():
    from hcache_deepspeed_amd.parallel.moe import MoE
    torch.manual_seed(0)
    H, I, E = 32, 48, 4
    moe = MoE(H, None, E, 1, k=2, capacity_factor=8.0, eval_capacity_factor=8.0, expert_intermediate_size=I)
    x = torch.randn(2, 9, H, requires_grad=True)
    out, l_aux, counts = moe(x)
    ex = moe.deepspeed_moe.experts
    wg = moe.deepspeed_moe.gate.wg.weight
    xr = x.detach().clone().requires_grad_(True)
    w13 = ex.w13.detach().clone().requires_grad_(True)
    w2 = ex.w2.detach().clone().requires_grad_(True)
    ref = _dense_moe_ref(xr.reshape(-1, H), wg.detach(), w13, w2, 2).view_as(x)
    assert torch.allclose(out, ref, atol=1e-5, rtol=1e-4)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    (ref * g).sum().backward()
    assert torch.allclose(x.grad, xr.grad, atol=1e-5, rtol=1e-4)
    assert torch.allclose(ex.w13.grad, w13.grad, atol=1e-5, rtol=1e-4)
    assert torch.allclose(ex.w2.grad, w2.grad, atol=1e-5, rtol=1e-4)
    assert wg.grad is not None and wg.grad.abs().sum() > 0  # router learns through the combine weights


def test_moe_capacity_drops_tokens():
    from hcache_deepspeed_amd.ops.moe import moe_combine, moe_dispatch, topk_route
    torch.manual_seed(1)
    T, H, E = 16, 8, 2
    x = torch.randn(T, H)
    logits = torch.zeros(T, E)
    logits[:, 0] = 5.0  # everyone wants expert 0
    expert, pos, w, C, _, _ = topk_route(logits, 1, capacity_factor=0.5, min_capacity=1)
    assert C == 4
    d = moe_dispatch(x, expert, pos, E, C)
    assert torch.equal(d[:C], x[:C])  # first C tokens kept, in order
    y = moe_combine(d, expert, pos, w, C)
    assert torch.allclose(y[:C], x[:C] * w[:C, :1]) and torch.all(y[C:] == 0)


def test_moe_generic_experts_module():
    import torch.nn as nn
    from hcache_deepspeed_amd.parallel.moe import MoE, is_moe_param, split_params_into_different_moe_groups_for_optimizer
    torch.manual_seed(0)
    moe = MoE(16, nn.Sequential(nn.Linear(16, 32), nn.GELU(), nn.Linear(32, 16)), num_experts=3, k=1,
              capacity_factor=4.0)
    x = torch.randn(5, 16)
    out, _, _ = moe(x)
    assert out.shape == x.shape
    # top-1: each token's output is its expert's output scaled by the gate prob
    probs = torch.softmax(x @ moe.deepspeed_moe.gate.wg.weight.t(), -1)
    p, e = probs.max(-1)
    for t in range(5):
        ref = moe.deepspeed_moe.experts.deepspeed_experts[int(e[t])](x[t]) * p[t]
        assert torch.allclose(out[t], ref, atol=1e-5)
    groups_ = split_params_into_different_moe_groups_for_optimizer({"params": list(moe.parameters()), "lr": 1.0})
    assert len(groups_) == 2 and groups_[1]["moe"] and all(is_moe_param(p) for p in groups_[1]["params"])


def _ep_exact(rank, world):
    from hcache_deepspeed_amd.parallel.moe import MoE
    H, I, E = 16, 24, 4
    torch.manual_seed(0)
    full_w13 = torch.randn(E, 2 * I, H) * 0.2
    full_w2 = torch.randn(E, H, I) * 0.2
    wg = torch.randn(E, H)
    moe = MoE(H, None, E, ep_size=2, k=2, capacity_factor=16.0, eval_capacity_factor=16.0,
              expert_intermediate_size=I)
    ex = moe.deepspeed_moe.experts
    assert ex.num_local_experts == 2
    with torch.no_grad():
        ex.w13.copy_(full_w13[2 * rank:2 * rank + 2])
        ex.w2.copy_(full_w2[2 * rank:2 * rank + 2])
        moe.deepspeed_moe.gate.wg.weight.copy_(wg)
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(7, H, generator=g)
    out, _, _ = moe(x)
    # reference: all experts locally
    w13 = full_w13.clone().requires_grad_(True)
    w2 = full_w2.clone().requires_grad_(True)
    ref = _dense_moe_ref(x, wg, w13, w2, 2)
    assert torch.allclose(out, ref, atol=1e-5, rtol=1e-4), (out - ref).abs().max()
    # expert grads: local experts see every rank's tokens through the all-to-all
    out.sum().backward()
    refs_all = []
    for r in range(world):
        xr = torch.randn(7, H, generator=torch.Generator().manual_seed(100 + r))
        refs_all.append(_dense_moe_ref(xr, wg, w13, w2, 2).sum())
    sum(refs_all).backward()
    assert torch.allclose(ex.w13.grad, w13.grad[2 * rank:2 * rank + 2], atol=1e-4, rtol=1e-4)
    assert torch.allclose(ex.w2.grad, w2.grad[2 * rank:2 * rank + 2], atol=1e-4, rtol=1e-4)


def test_expert_parallel_all_to_all_exact():
    run_distributed(_ep_exact, 2)


TINY_MOE = dict(head_dim=16, hidden_size=32, intermediate_size=48, vocab_size=97, num_attention_heads=2,
                num_key_value_heads=1, num_hidden_layers=2, num_local_experts=4, num_experts_per_tok=2,
                capacity_factor=8.0)


def _mixtral_stages(rank, world, ep):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.mixtral import MixtralForCausalLM, tiny_moe
    from hcache_deepspeed_amd.utils import groups
    g = torch.Generator().manual_seed(5 + rank)
    batches = [torch.randint(0, 97, (2, 12), generator=g) for _ in range(3)]
    results = {}
    for stage in (0, 1, 2, 3):
        torch.manual_seed(0)
        m = MixtralForCausalLM(tiny_moe(ep_size=ep, **TINY_MOE))
        ep_rank = torch.distributed.get_rank(groups._get_expert_parallel_group(f"ep_size_{ep}"))
        gen = torch.Generator().manual_seed(1000 + ep_rank)
        with torch.no_grad():
            for layer in m.layers:
                ex = layer.block_sparse_moe.deepspeed_moe.experts
                ex.w13.copy_(torch.randn(ex.w13.shape, generator=gen) * 0.05)
                ex.w2.copy_(torch.randn(ex.w2.shape, generator=gen) * 0.05)
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
               "zero_optimization": {"stage": stage}, "gradient_clipping": 0.3}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        zopt = eng.optimizer
        assert len(zopt.expert_units) >= 1
        for u in zopt.expert_units:
            assert u.world == (1 if stage == 0 else world // ep)
        losses = []
        for b in batches:
            loss = eng(b, labels=b)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
        results[stage] = (losses, eng.get_global_grad_norm())
    base = results[0]
    for stage, (losses, norm) in results.items():
        assert losses == pytest.approx(base[0], rel=2e-4, abs=2e-4), (stage, losses, base[0])
        assert norm == pytest.approx(base[1], rel=1e-3), (stage, norm, base[1])
    # the EP ranks really hold different experts and dense params stay replicated
    assert results[0][0][-1] < results[0][0][0] + 1.0


@pytest.mark.parametrize("world,ep", [(2, 2), (4, 2)])
def test_mixtral_zero_stages_with_expert_parallel(world, ep):
    run_distributed(_mixtral_stages, world, ep)


def _moe_ckpt(rank, world, ep, stage, d):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.checkpoint.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
    from hcache_deepspeed_amd.models.mixtral import MixtralForCausalLM, tiny_moe
    from hcache_deepspeed_amd.utils import groups

    def build():
        torch.manual_seed(0)
        m = MixtralForCausalLM(tiny_moe(ep_size=ep, **TINY_MOE))
        ep_rank = torch.distributed.get_rank(groups._get_expert_parallel_group(f"ep_size_{ep}"))
        with torch.no_grad():
            for layer in m.layers:
                layer.block_sparse_moe.deepspeed_moe.experts.w13.add_(ep_rank * 0.01)
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
               "zero_optimization": {"stage": stage}}
        return ds.initialize(model=m, config=cfg)[0]

    g = torch.Generator().manual_seed(5 + rank)
    batches = [torch.randint(0, 97, (2, 12), generator=g) for _ in range(4)]
    eng = build()
    for b in batches[:2]:
        eng.backward(eng(b, labels=b))
        eng.step()
    eng.save_checkpoint(d, tag="t")
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    ref_losses = []
    for b in batches[2:]:
        loss = eng(b, labels=b)
        eng.backward(loss)
        eng.step()
        ref_losses.append(float(loss))
    eng2 = build()
    eng2.load_checkpoint(d, tag="t")
    losses = []
    for b in batches[2:]:
        loss = eng2(b, labels=b)
        eng2.backward(loss)
        eng2.step()
        losses.append(float(loss))
    assert losses == pytest.approx(ref_losses, rel=1e-5, abs=1e-5)
    torch.distributed.barrier()
    if rank == 0:
        sd = get_fp32_state_dict_from_zero_checkpoint(d, tag="t")
        k = "layers.0.block_sparse_moe.deepspeed_moe.experts.w13"
        assert sd[k].shape[0] == TINY_MOE["num_local_experts"]
        assert set(sd) == set(full)
        for n in sd:
            assert torch.allclose(sd[n], full[n]), n


@pytest.mark.parametrize("stage", [0, 2, 3])
def test_moe_checkpoint_roundtrip_and_consolidation(tmp_path, stage):
    run_distributed(_moe_ckpt, 4, 2, stage, str(tmp_path))


def _expert_tp(rank, world, cf):
    """EP=2 x expert-TP=2 on 4 ranks (TP dense model: tokens replicated over each TP pair) against the unsharded
    MoE run on every data-parallel rank's tokens."""
    from hcache_deepspeed_amd.parallel.moe import MoE
    from hcache_deepspeed_amd.utils import groups
    groups.initialize(tp=2)
    tp_rank, dp_rank = groups.get_tensor_model_parallel_rank(), groups.get_data_parallel_rank()
    H, I, E, T = 16, 24, 4, 7
    torch.manual_seed(0)
    full_w13 = torch.randn(E, 2 * I, H) * 0.2
    full_w2 = torch.randn(E, H, I) * 0.2
    wg = torch.randn(E, H)
    kw = dict(k=2, capacity_factor=cf, eval_capacity_factor=cf, min_capacity=1, use_rts=False,
              expert_intermediate_size=I)
    moe = MoE(H, None, E, ep_size=2, enable_expert_tensor_parallelism=True, **kw)
    ex = moe.deepspeed_moe.experts
    assert moe.enable_expert_tensor_parallelism and ex.tp_size == 2 and ex.w2.shape == (2, H, I // 2)
    ep_rank = dp_rank  # EP groups pair ranks of equal TP coordinate
    ex.load_full(full_w13[2 * ep_rank:2 * ep_rank + 2], full_w2[2 * ep_rank:2 * ep_rank + 2], tp_rank)
    with torch.no_grad():
        moe.deepspeed_moe.gate.wg.weight.copy_(wg)
    xs = [torch.randn(T, H, generator=torch.Generator().manual_seed(100 + d)) for d in range(2)]
    x = xs[dp_rank].clone().requires_grad_(True)
    out, _, _ = moe(x)
    out.sum().backward()

    ref = MoE(H, None, E, ep_size=1, **kw)
    with torch.no_grad():
        ref.deepspeed_moe.experts.w13.copy_(full_w13)
        ref.deepspeed_moe.experts.w2.copy_(full_w2)
        ref.deepspeed_moe.gate.wg.weight.copy_(wg)
    xr = [t.clone().requires_grad_(True) for t in xs]
    outs = [ref(t)[0] for t in xr]
    assert torch.allclose(out, outs[dp_rank], atol=1e-5, rtol=1e-4), (out - outs[dp_rank]).abs().max()
    sum(o.sum() for o in outs).backward()
    assert torch.allclose(x.grad, xr[dp_rank].grad, atol=1e-5, rtol=1e-4)
    probe = GroupedSwiGLUExperts_shard(ref.deepspeed_moe.experts, 2 * ep_rank, tp_rank)
    assert torch.allclose(ex.w13.grad, probe[0], atol=1e-4, rtol=1e-4)
    assert torch.allclose(ex.w2.grad, probe[1], atol=1e-4, rtol=1e-4)


def GroupedSwiGLUExperts_shard(full, e0, tp_rank, tp=2):
    """This (EP, TP) rank's slice of the unsharded experts' weight gradients."""
    I = full.w2.shape[-1]
    i = I // tp
    lo = tp_rank * i
    g13 = full.w13.grad[e0:e0 + 2]
    return (torch.cat([g13[:, lo:lo + i], g13[:, I + lo:I + lo + i]], 1), full.w2.grad[e0:e0 + 2, :, lo:lo + i])


@pytest.mark.parametrize("cf", [16.0, 0.6])  # no drops / drops with a capacity padded to the TP size
def test_expert_tensor_parallel_matches_unsharded(cf):
    run_distributed(_expert_tp, 4, cf)


def test_moe_experts_skip_empty_capacity_slots(monkeypatch):
    """The grouped experts run their GEMMs over each expert's occupied capacity slots only (rounded up to 128
    rows) and zero the rest: outputs and gradients match running every slot."""
    import hcache_deepspeed_amd.parallel.moe as M
    torch.manual_seed(3)
    H, I, E, T = 16, 24, 4, 600
    res = {}
    real = M._ExpertLinear.forward
    calls = []
    monkeypatch.setattr(M._ExpertLinear, "forward",
                        staticmethod(lambda ctx, a, w, rows=None: calls.append(rows) or real(ctx, a, w, rows)))
    for exact in (True, False):
        monkeypatch.setattr(M, "_EXACT_ROWS", exact)
        calls.clear()
        torch.manual_seed(3)
        moe = M.MoE(H, None, E, 1, k=2, capacity_factor=2.0, eval_capacity_factor=2.0, expert_intermediate_size=I)
        x = torch.randn(T, H, requires_grad=True)
        out, _, counts = moe(x)
        (out * torch.linspace(-1, 1, out.numel()).view_as(out)).sum().backward()
        ex = moe.deepspeed_moe.experts
        res[exact] = (out.detach(), x.grad, ex.w13.grad, ex.w2.grad)
        if exact:
            C = 600  # ceil(T * k / E * capacity_factor)
            ms = [m for seg in calls[0] for _, m in seg]
            assert calls[0] is not None and all(m % 128 == 0 or m == C for m in ms)
            assert max(ms) < C  # the path skipped empty slots
        else:
            assert calls[0] is None
    for a, b in zip(res[True], res[False]):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


def _ep_segments(rank, world):
    import hcache_deepspeed_amd.parallel.moe as M
    H, I, E, T = 16, 24, 4, 600
    res = {}
    seen = []
    real = M.occupied_segments
    M.occupied_segments = lambda *a, **k: seen.append(real(*a, **k)) or seen[-1]
    try:
        for exact in (True, False):
            M._EXACT_ROWS = exact
            torch.manual_seed(3)
            moe = M.MoE(H, None, E, ep_size=2, k=2, capacity_factor=2.0, eval_capacity_factor=2.0,
                        expert_intermediate_size=I)
            x = torch.randn(T, H, generator=torch.Generator().manual_seed(50 + rank), requires_grad=True)
            out, _, _ = moe(x)
            (out * torch.linspace(-1, 1, out.numel()).view_as(out)).sum().backward()
            ex = moe.deepspeed_moe.experts
            res[exact] = (out.detach(), x.grad, ex.w13.grad, ex.w2.grad)
    finally:
        M.occupied_segments = real
        M._EXACT_ROWS = True
    # one segment per source rank for each of the 2 local experts, each a rounded prefix of its 600-row block
    assert len(seen) == 1 and all(len(s) == 2 for s in seen[0])
    assert all(s0 % 600 == 0 and m % 128 == 0 and m < 600 for s in seen[0] for s0, m in s)
    for a, b in zip(res[True], res[False]):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


def test_expert_parallel_skips_empty_slots_per_source_rank():
    run_distributed(_ep_segments, 2)
