"""Block-sparse attention: layouts, compressed-format MatMul/Softmax, SparseSelfAttention, and the fused HIP kernel.

Reference test analogue: tests/unit/ops/sparse_attention/test_sparse_attention.py (sdd/dsd/dds matmul and
softmax against dense torch references with the layout expanded to a dense mask; SparseSelfAttention vs dense
attention). Numerics reference here: plain fp32 torch attention with the block layout as a dense mask.
"""
import math

import pytest
import torch

from hcache_deepspeed_amd.ops.sparse_attention import (BigBirdSparsityConfig, BSLongformerSparsityConfig,
                                                       DenseSparsityConfig, FixedSparsityConfig,
                                                       LocalSlidingWindowSparsityConfig, MatMul, Softmax,
                                                       SparseSelfAttention, VariableSparsityConfig,
                                                       block_sparse_attention)


def _dense_mask(layout, block):
    return layout.repeat_interleave(block, 1).repeat_interleave(block, 2).bool()


def _ref_attn(q, k, v, mask, scale, causal=False):
    G = q.shape[1] // k.shape[1]
    k = k.float().repeat_interleave(G, 1)
    v = v.float().repeat_interleave(G, 1)
    s = torch.matmul(q.float(), k.transpose(-1, -2)) * scale
    m = mask.to(q.device)
    if causal:
        S = q.shape[2]
        m = m & torch.tril(torch.ones(S, S, dtype=torch.bool, device=q.device))
    s = s.masked_fill(~m, float("-inf"))
    p = torch.softmax(s, -1).nan_to_num(0.0)
    return torch.matmul(p, v)


@pytest.mark.parametrize("cfg", [
    DenseSparsityConfig(num_heads=2, block=16),
    FixedSparsityConfig(num_heads=2, block=16, num_local_blocks=4, num_global_blocks=1),
    FixedSparsityConfig(num_heads=4, block=16, different_layout_per_head=True, num_local_blocks=4,
                        num_global_blocks=1, attention="unidirectional", num_different_global_patterns=2),
    VariableSparsityConfig(num_heads=2, block=16, num_random_blocks=1, local_window_blocks=[2, 4],
                           global_block_indices=[0]),
    BigBirdSparsityConfig(num_heads=2, block=16, num_random_blocks=1, num_sliding_window_blocks=3),
    BSLongformerSparsityConfig(num_heads=2, block=16, num_sliding_window_blocks=3, global_block_indices=[0]),
    LocalSlidingWindowSparsityConfig(num_heads=2, block=16, num_sliding_window_blocks=3),
])
def test_layouts(cfg):
    lay = cfg.make_layout(128)
    assert lay.shape == (cfg.num_heads, 8, 8)
    assert lay.dtype == torch.int64 and int(lay.max()) <= 1
    assert bool((lay.sum(-1) > 0).all()), "every query block must attend somewhere"
    if getattr(cfg, "attention", "bidirectional") == "unidirectional":
        assert torch.equal(lay, torch.tril(lay))
    if not cfg.different_layout_per_head:
        assert all(torch.equal(lay[0], lay[h]) for h in range(cfg.num_heads))
    if isinstance(cfg, BigBirdSparsityConfig):
        assert bool(lay[:, 0, :].all()) and bool(lay[:, :, 0].all())
    with pytest.raises(ValueError):
        cfg.make_layout(100)


def test_matmul_modes_and_softmax_match_dense():
    torch.manual_seed(0)
    B, H, S, D, blk = 2, 2, 64, 8, 16
    lay = BigBirdSparsityConfig(num_heads=H, block=blk, different_layout_per_head=True).make_layout(S)
    mask = _dense_mask(lay, blk)
    a, b = torch.randn(B, H, S, D), torch.randn(B, H, S, D)
    sdd = MatMul(lay, blk, "sdd", trans_b=True)
    comp = sdd(a, b)  # [B, nnz, blk, blk]
    dense = torch.matmul(a, b.transpose(-1, -2))
    nz = lay.nonzero()
    for e, (h, r, c) in enumerate(nz.tolist()):
        assert torch.allclose(comp[:, e], dense[:, h, r * blk:(r + 1) * blk, c * blk:(c + 1) * blk], atol=1e-5)
    sm = Softmax(lay, blk)
    p = sm(comp, scale=0.5)
    ref = torch.softmax((dense * 0.5).masked_fill(~mask, float("-inf")), -1)
    dsd = MatMul(lay, blk, "dsd")
    v = torch.randn(B, H, S, D)
    assert torch.allclose(dsd(p, v), ref @ v, atol=1e-5)
    dds = MatMul(lay, blk, "dds")
    x = torch.randn(B, H, D, S)
    assert torch.allclose(dds(x, p), x @ ref, atol=1e-5)


def test_sparse_self_attention_with_masks_and_rpe():
    torch.manual_seed(1)
    B, H, S, D, blk = 2, 4, 64, 16, 16
    cfg = FixedSparsityConfig(num_heads=H, block=blk, num_local_blocks=2, num_global_blocks=1)
    attn = SparseSelfAttention(cfg, key_padding_mask_mode="add", attn_mask_mode="mul")
    q, k, v = (torch.randn(B, H, S, D, requires_grad=True) for _ in range(3))
    kpm = torch.zeros(B, S)
    kpm[1, -5:] = float("-inf")
    am = torch.ones(S, S)
    am[3, 1] = 0
    rpe = torch.randn(H, S, S) * 0.1
    out = attn(q, k, v, rpe=rpe, key_padding_mask=kpm, attn_mask=am)
    mask = _dense_mask(attn.get_layout(S), blk)
    s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(D) + rpe[None] + kpm[:, None, None, :]
    s = s.masked_fill(~mask[None] | (am == 0)[None, None], float("-inf"))
    ref = torch.softmax(s, -1) @ v
    assert torch.allclose(out, ref, atol=1e-5)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, (q, k, v), g)
    gb = torch.autograd.grad(ref, (q, k, v), g)
    for x, y in zip(ga, gb):
        assert torch.allclose(x, y, atol=1e-4)


def test_block_sparse_attention_causal_gqa_cpu():
    torch.manual_seed(2)
    B, Hq, Hkv, S, D, blk = 1, 4, 2, 64, 16, 16
    lay = BSLongformerSparsityConfig(num_heads=1, block=blk, num_sliding_window_blocks=3).make_layout(S)
    q = torch.randn(B, Hq, S, D)
    k, v = torch.randn(B, Hkv, S, D), torch.randn(B, Hkv, S, D)
    out = block_sparse_attention(q, k, v, lay, blk, causal=True)
    ref = _ref_attn(q, k, v, _dense_mask(lay, blk)[0], 1 / math.sqrt(D), causal=True)
    assert torch.allclose(out, ref, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("block,causal,hkv,per_head", [(64, False, 4, False), (64, True, 2, False),
                                                        (128, True, 4, True), (64, False, 1, True)])
def test_block_sparse_attention_hip(block, causal, hkv, per_head):
    """Fused HIP kernel (sparse_attn.hip) fwd + bwd vs fp32 dense-masked attention."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(3)
    dev = torch.device("cuda")
    B, Hq, S, D = 2, 4, 1024, 128
    cfg = BigBirdSparsityConfig(num_heads=Hq, block=block, different_layout_per_head=per_head, num_random_blocks=2,
                                num_sliding_window_blocks=3)
    lay = cfg.make_layout(S)
    lay_k = lay if per_head else lay[:1]
    q = torch.randn(B, Hq, S, D, device=dev).bfloat16().requires_grad_(True)
    k = torch.randn(B, hkv, S, D, device=dev).bfloat16().requires_grad_(True)
    v = torch.randn(B, hkv, S, D, device=dev).bfloat16().requires_grad_(True)
    out = block_sparse_attention(q, k, v, lay_k, block, causal=causal)
    mask = _dense_mask(lay, block).to(dev)
    if not per_head:
        mask = mask[:1]
    qf, kf, vf = (x.detach().float().requires_grad_(True) for x in (q, k, v))
    ref = _ref_attn(qf, kf, vf, mask, 1 / math.sqrt(D), causal=causal)
    g = torch.randn_like(ref)
    gq, gk, gv = torch.autograd.grad(out, (q, k, v), g.bfloat16())
    rq, rk, rv = torch.autograd.grad(ref, (qf, kf, vf), g)
    torch.cuda.synchronize()

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-6)).item()

    assert rel(out, ref) < 1e-2
    assert rel(gq, rq) < 2e-2 and rel(gk, rk) < 2e-2 and rel(gv, rv) < 2e-2
