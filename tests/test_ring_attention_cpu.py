"""Ring attention (zigzag context parallelism) vs single-process dense attention.

The reference has no ring attention; parity target is the dense causal/full attention of
the same q/k/v: outputs and q/k/v gradients of every rank's zigzag shard must match the dense result.
"""
import torch

from tests.dist_utils import run_distributed


def _dense(q, k, v, causal):
    from hcache_deepspeed_amd.ops.attention import flash_attn
    return flash_attn(q, k, v, causal=causal)


def _ring_vs_dense(rank, world, causal):
    import torch.distributed as tdist
    from hcache_deepspeed_amd.parallel.ring_attention import ring_attention, zigzag_shard
    torch.manual_seed(0)
    B, S, Hq, Hkv, D = 2, 8 * world, 4, 2, 16
    q = torch.randn(B, S, Hq, D, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, requires_grad=True)
    do = torch.randn(B, S, Hq, D)
    o0 = _dense(q, k, v, causal)
    gq0, gk0, gv0 = torch.autograd.grad(o0, (q, k, v), do)

    group = tdist.new_group(list(range(world)))
    ql, kl, vl = (zigzag_shard(t.detach(), world, rank).requires_grad_(True) for t in (q, k, v))
    o = ring_attention(ql, kl, vl, group, causal=causal)
    assert torch.allclose(o, zigzag_shard(o0.detach(), world, rank), atol=1e-5), \
        (o - zigzag_shard(o0.detach(), world, rank)).abs().max()
    gq, gk, gv = torch.autograd.grad(o, (ql, kl, vl), zigzag_shard(do, world, rank))
    for g, g0 in ((gq, gq0), (gk, gk0), (gv, gv0)):
        ref = zigzag_shard(g0, world, rank)
        assert torch.allclose(g, ref, atol=1e-4), (g - ref).abs().max()


def test_ring_attention_causal_cp2():
    run_distributed(_ring_vs_dense, 2, True)


def test_ring_attention_causal_cp3():
    run_distributed(_ring_vs_dense, 3, True)


def test_ring_attention_full_cp2():
    run_distributed(_ring_vs_dense, 2, False)


def test_zigzag_roundtrip():
    from hcache_deepspeed_amd.parallel.ring_attention import zigzag_shard, zigzag_unshard
    x = torch.arange(2 * 24).view(2, 24)
    for P in (1, 2, 3, 4):
        shards = [zigzag_shard(x, P, r) for r in range(P)]
        assert torch.equal(zigzag_unshard(shards), x)
    # rank 0 of P=2 holds chunks 0 and 3
    assert zigzag_shard(x, 2, 0)[0].tolist() == list(range(0, 6)) + list(range(18, 24))
