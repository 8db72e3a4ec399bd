"""Tensor parallelism (AutoTP) and Ulysses sequence parallelism on gloo: must reproduce single-process training."""
import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


def _ref_losses(batches, steps, targets_mode=False):
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    ref = LlamaForCausalLM(tiny(**TINY))
    opt = torch.optim.AdamW(ref.parameters(), lr=5e-3)
    out = []
    for b in batches[:steps]:
        if targets_mode:
            x, t = b
            loss = ref(x, targets=t)
        else:
            loss = ref(b, labels=b)
        loss.backward()
        opt.step()
        opt.zero_grad()
        out.append(float(loss))
    return out, ref


def _tp(rank, world, stage):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    g = torch.Generator().manual_seed(7)
    batches = [torch.randint(0, 97, (2, 12), generator=g) for _ in range(3)]
    ref_losses, _ = _ref_losses(batches, 3)
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
           "zero_optimization": {"stage": stage}, "tensor_parallel": {"autotp_size": 2}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    assert m.model.layers[0].self_attn.n_q == TINY["num_attention_heads"] // 2
    losses = []
    for b in batches:
        loss = eng(b, labels=b)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    assert losses == pytest.approx(ref_losses, rel=1e-4, abs=1e-4), (losses, ref_losses)


@pytest.mark.parametrize("stage", [0, 3])
def test_autotp_training_matches_single(stage):
    from hcache_deepspeed_amd.utils import groups
    run_distributed(_tp, 2, stage)


def _sp(rank, world, stage, use_mesh=False):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    g = torch.Generator().manual_seed(9)
    S = 16
    batches = []
    for _ in range(3):
        x = torch.randint(0, 97, (2, S + 1), generator=g)
        x, t = x[:, :-1].contiguous(), x[:, 1:].contiguous()  # every position valid: equal counts per rank
        batches.append((x, t))
    ref_losses, ref = _ref_losses(batches, 3, targets_mode=True)
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
           "zero_optimization": {"stage": stage}, "sequence_parallel_size": 2}
    if use_mesh:  # the same layout requested through initialize(mesh_param=(dp, sp))
        del cfg["sequence_parallel_size"]
        eng, _, _, _ = ds.initialize(model=m, config=cfg, mesh_param=(1, 2))
    else:
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
    half = S // 2
    losses = []
    for x, t in batches:
        xs, ts = x[:, rank * half:(rank + 1) * half], t[:, rank * half:(rank + 1) * half]
        loss = eng(xs, targets=ts)
        eng.backward(loss)
        eng.step()
        lt = loss.detach().clone()
        ds.comm.all_reduce(lt)
        losses.append(float(lt) / 2)
    assert losses == pytest.approx(ref_losses, rel=1e-4, abs=1e-4), (losses, ref_losses)
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    for n, p in ref.named_parameters():
        assert torch.allclose(full[n], p.detach(), atol=2e-4), n


@pytest.mark.parametrize("stage", [1, 3])
def test_ulysses_sp_matches_single(stage):
    run_distributed(_sp, 2, stage)


def test_mesh_param_sets_sequence_parallel():
    run_distributed(_sp, 2, 3, True)


def _ulysses_a2a(rank, world):
    from hcache_deepspeed_amd.parallel.ulysses import DistributedAttention
    from hcache_deepspeed_amd.utils import groups
    groups.initialize(sp=2)
    grp = groups._get_sequence_parallel_group()
    torch.manual_seed(0)
    B, S, H, D = 2, 8, 4, 16
    q, k, v = (torch.randn(B, S, H, D) for _ in range(3))

    def local(q_, k_, v_):
        return torch.nn.functional.scaled_dot_product_attention(q_.transpose(1, 2), k_.transpose(1, 2),
                                                                v_.transpose(1, 2), is_causal=True).transpose(1, 2)

    full = local(q, k, v)
    sl = slice(rank * S // 2, (rank + 1) * S // 2)
    da = DistributedAttention(local, grp)
    out = da(q[:, sl].contiguous(), k[:, sl].contiguous(), v[:, sl].contiguous())
    assert torch.allclose(out, full[:, sl], atol=1e-5)


def test_distributed_attention_api():
    run_distributed(_ulysses_a2a, 2)


def _domino(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.parallel.domino import enable_domino
    g = torch.Generator().manual_seed(11)
    batches = [torch.randint(0, 97, (4, 12), generator=g) for _ in range(3)]
    ref_losses, _ = _ref_losses(batches, 3)
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
           "zero_optimization": {"stage": 1}, "tensor_parallel": {"autotp_size": 2}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    enable_domino(m)
    assert m.model._domino_group is not None
    losses = []
    for b in batches:
        loss = eng(b, labels=b)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    assert losses == pytest.approx(ref_losses, rel=1e-4, abs=1e-4), (losses, ref_losses)


def test_domino_tp_matches_single():
    """Domino half-batch overlap of the TP all-reduces reproduces single-process training."""
    run_distributed(_domino, 2)


def _gqa_local(q_, k_, v_):
    """[B, S, Hq, D] x [B, S, Hkv, D] causal attention; q head i uses kv head i // (Hq // Hkv)."""
    G = q_.shape[2] // k_.shape[2]
    k_ = k_.repeat_interleave(G, dim=2)
    v_ = v_.repeat_interleave(G, dim=2)
    return torch.nn.functional.scaled_dot_product_attention(q_.transpose(1, 2), k_.transpose(1, 2),
                                                            v_.transpose(1, 2), is_causal=True).transpose(1, 2)


def _ulysses_uneven(rank, world, n_q, n_kv):
    import hcache_deepspeed_amd.comm as hcomm
    from hcache_deepspeed_amd.parallel.ulysses import DistributedAttention
    from hcache_deepspeed_amd.utils import groups
    groups.initialize(sp=world)
    grp = groups._get_sequence_parallel_group()
    torch.manual_seed(0)
    B, S, D = 2, 16, 8
    q = torch.randn(B, S, n_q, D, requires_grad=True)
    k = torch.randn(B, S, n_kv, D, requires_grad=True)
    v = torch.randn(B, S, n_kv, D, requires_grad=True)
    go = torch.randn(B, S, n_q, D)
    full = _gqa_local(q, k, v)
    full.backward(go)
    sl = slice(rank * S // world, (rank + 1) * S // world)
    ql, kl, vl = (t.detach()[:, sl].clone().requires_grad_(True) for t in (q, k, v))
    # record the order of all-to-all issues and waits: with even heads all three must be in flight before a wait
    log, orig = [], hcomm.all_to_all_single

    class W:
        def __init__(self, w):
            self.w = w

        def wait(self):
            log.append("wait")
            return self.w.wait() if self.w is not None else True

    def spy(*a, async_op=False, **kw):
        log.append("issue")
        w = orig(*a, async_op=async_op, **kw)
        return W(w) if async_op else w

    hcomm.all_to_all_single = spy
    try:
        out = DistributedAttention(_gqa_local, grp, sp_stream=object())(ql, kl, vl)
    finally:
        hcomm.all_to_all_single = orig
    assert torch.allclose(out, full[:, sl], atol=1e-5), (out - full[:, sl]).abs().max()
    out.backward(go[:, sl])
    for a, b in ((ql, q), (kl, k), (vl, v)):
        assert torch.allclose(a.grad, b.grad[:, sl], atol=1e-5), (a.grad - b.grad[:, sl]).abs().max()
    if n_q % world == 0 and n_kv % world == 0:
        assert log[:4] == ["issue", "issue", "issue", "wait"], log


@pytest.mark.parametrize("heads", [(6, 2), (8, 4), (7, 7)])
def test_ulysses_uneven_heads_and_gqa_world4(heads):
    """6 q / 2 kv heads on 4 ranks (kv heads replicated, uneven q split), 7 heads on 4 ranks (uneven MHA), and the
    even case with its three all-to-alls issued before the first wait; forward and backward match unsharded."""
    run_distributed(_ulysses_uneven, 4, *heads)


def _sp_llama_uneven(rank, world):
    """The Llama attention path (fused qkv all-to-all) with 6 q / 2 kv heads at sp = 4: loss and gradients match
    one process."""
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.parallel.ulysses import enable_sequence_parallel
    from hcache_deepspeed_amd.utils import groups
    groups.initialize(sp=world)
    grp = groups._get_sequence_parallel_group()
    cfg = dict(vocab_size=64, hidden_size=48, intermediate_size=64, num_hidden_layers=2, num_attention_heads=6,
               num_key_value_heads=2, head_dim=8, max_position_embeddings=64)
    torch.manual_seed(0)
    ref = LlamaForCausalLM(tiny(**cfg))
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**cfg))
    enable_sequence_parallel(m, grp)
    g = torch.Generator().manual_seed(5)
    S = 16
    x = torch.randint(0, 64, (2, S + 1), generator=g)
    x, t = x[:, :-1].contiguous(), x[:, 1:].contiguous()
    lr = ref(x, targets=t)
    lr.backward()
    sl = slice(rank * S // world, (rank + 1) * S // world)
    loss = m(x[:, sl].contiguous(), targets=t[:, sl].contiguous())
    loss.backward()
    lt = loss.detach().clone()
    torch.distributed.all_reduce(lt)
    assert abs(float(lt) / world - float(lr)) < 1e-4
    for (n, p), (_, pr) in zip(m.named_parameters(), ref.named_parameters()):
        gsum = p.grad.clone()
        torch.distributed.all_reduce(gsum)
        assert torch.allclose(gsum / world, pr.grad, atol=1e-5, rtol=1e-3), (n, (gsum / world - pr.grad).abs().max())


def test_ulysses_llama_gqa_fewer_kv_heads_than_ranks():
    run_distributed(_sp_llama_uneven, 4)


def _sp_ce(rank, world):
    from hcache_deepspeed_amd.sequence.cross_entropy import vocab_sequence_parallel_cross_entropy
    from hcache_deepspeed_amd.utils import groups
    groups.initialize(sp=world)
    grp = groups._get_sequence_parallel_group()
    torch.manual_seed(0)
    S, B, V = 8, 3, 11
    logits = torch.randn(S, B, V, requires_grad=True)
    target = torch.randint(0, V, (S, B))
    ref = torch.nn.functional.cross_entropy(logits.view(-1, V), target.view(-1), reduction="none").view(S, B)
    gout = torch.randn(S, B)
    ref.backward(gout)
    sl = slice(rank * S // world, (rank + 1) * S // world)
    mine = logits.detach()[sl].clone().requires_grad_(True)
    loss = vocab_sequence_parallel_cross_entropy(mine, target[sl], grp)
    assert loss.shape == (S, B) and torch.allclose(loss, ref.detach(), atol=1e-5)
    loss.backward(gout)
    assert torch.allclose(mine.grad, logits.grad[sl], atol=1e-5)


def test_vocab_sequence_parallel_cross_entropy():
    run_distributed(_sp_ce, 2)
