"""CPU (reference-path) checks of the op wrappers: autograd plumbing, shapes, math."""
import math

import torch

from hcache_deepspeed_amd.ops.activations import glu
from hcache_deepspeed_amd.ops.attention import flash_attn, qkv_attention
from hcache_deepspeed_amd.ops.cross_entropy import cross_entropy, fused_linear_cross_entropy
from hcache_deepspeed_amd.ops.norm import layer_norm, rms_norm
from hcache_deepspeed_amd.ops.optimizers import FusedAdam, adam_flat, clip_coef, grad_sumsq
from hcache_deepspeed_amd.ops.rope import apply_rotary, rope_, rope_tables


def test_rmsnorm_grad_matches_autograd():
    torch.manual_seed(0)
    x = torch.randn(5, 16, dtype=torch.float64, requires_grad=True)
    r = torch.randn(5, 16, dtype=torch.float64, requires_grad=True)
    w = torch.randn(16, dtype=torch.float64, requires_grad=True)
    y, h = rms_norm(x.float(), w.float(), 1e-6, residual=r.float())
    xr, rr, wr = (t.detach().clone().requires_grad_(True) for t in (x, r, w))
    hr = xr + rr
    yr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-6) * wr
    assert torch.allclose(y.double(), yr, atol=1e-5)
    gy, gh = torch.randn_like(yr), torch.randn_like(yr)
    torch.autograd.backward([y, h], [gy.float(), gh.float()])
    torch.autograd.backward([yr, hr], [gy, gh])
    assert torch.allclose(x.grad, xr.grad, atol=1e-4)
    assert torch.allclose(r.grad, rr.grad, atol=1e-4)
    assert torch.allclose(w.grad, wr.grad, atol=1e-4)


def test_layernorm_cpu():
    x = torch.randn(7, 32, requires_grad=True)
    w = torch.randn(32, requires_grad=True)
    b = torch.randn(32, requires_grad=True)
    y = layer_norm(x, w, b)
    ref = torch.nn.functional.layer_norm(x, (32, ), w, b)
    assert torch.allclose(y, ref, atol=1e-5)
    g = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), g)
    rx, rw, rb = torch.autograd.grad(ref, (x, w, b), g)
    assert torch.allclose(gx, rx, atol=1e-4) and torch.allclose(gw, rw, atol=1e-4) and torch.allclose(gb, rb, atol=1e-4)


def test_rope_roundtrip_cpu():
    cos, sin = rope_tables(64, 16, 10000.0)
    x = torch.randn(20, 3, 16)
    y = x.clone()
    rope_(y, cos, sin, 2, seq_len=10)
    assert not torch.allclose(y[:, :2], x[:, :2])
    assert torch.equal(y[:, 2], x[:, 2])
    rope_(y, cos, sin, 2, seq_len=10, sign=-1.0)
    assert torch.allclose(y, x, atol=1e-5)
    xa = x.clone().requires_grad_(True)
    out = apply_rotary(xa, cos, sin, seq_len=10)
    out.sum().backward()
    assert xa.grad.shape == x.shape


def test_llama3_rope_scaling():
    from hcache_deepspeed_amd.ops.rope import rope_inv_freq
    inv = rope_inv_freq(128, 500000.0, {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                        "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    base = rope_inv_freq(128, 500000.0)
    assert inv.shape == (64, ) and torch.all(inv <= base + 1e-12)
    assert torch.allclose(inv[:8], base[:8])  # high-frequency dims unchanged


def test_glu_cpu_grad():
    gu = torch.randn(4, 2 * 8, dtype=torch.float64, requires_grad=True)
    y = glu(gu.float(), "silu")
    g, u = gu.split(8, -1)
    ref = torch.nn.functional.silu(g) * u
    assert torch.allclose(y.double(), ref, atol=1e-5)
    (dy, ) = torch.autograd.grad(y.sum(), gu)
    (dr, ) = torch.autograd.grad(ref.sum(), gu)
    assert torch.allclose(dy, dr, atol=1e-4)


def test_attention_cpu_reference_paths():
    B, S, Hq, Hkv, D = 2, 12, 4, 2, 16
    q = torch.randn(B, S, Hq, D, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, requires_grad=True)
    o = flash_attn(q, k, v, causal=True)
    kk = k.repeat_interleave(2, 2).transpose(1, 2)
    vv = v.repeat_interleave(2, 2).transpose(1, 2)
    ref = torch.nn.functional.scaled_dot_product_attention(q.transpose(1, 2), kk, vv, is_causal=True).transpose(1, 2)
    assert torch.allclose(o, ref, atol=1e-5)
    g = torch.randn_like(o)
    a = torch.autograd.grad(o, (q, k, v), g)
    b = torch.autograd.grad(ref, (q, k, v), g)
    for x, y in zip(a, b):
        assert torch.allclose(x, y, atol=1e-4)
    # fused qkv path
    cos, sin = rope_tables(S, D, 10000.0)
    qkv = torch.randn(B * S, Hq + 2 * Hkv, D, requires_grad=True)
    out = qkv_attention(qkv.clone(), Hq, Hkv, cos, sin, seq_len=S)
    out.sum().backward()
    assert out.shape == (B * S, Hq * D) and qkv.grad.shape == qkv.shape


def test_cross_entropy_cpu():
    logits = torch.randn(9, 11, requires_grad=True)
    t = torch.randint(0, 11, (9, ))
    t[0] = -100
    loss = cross_entropy(logits, t)
    ref = torch.nn.functional.cross_entropy(logits, t)
    assert torch.allclose(loss, ref, atol=1e-6)
    h = torch.randn(9, 6, requires_grad=True)
    w = torch.randn(11, 6, requires_grad=True)
    l2 = fused_linear_cross_entropy(h, w, t, chunk_rows=4)
    r2 = torch.nn.functional.cross_entropy(h @ w.t(), t)
    assert torch.allclose(l2, r2, atol=1e-5)
    ga = torch.autograd.grad(3 * l2, (h, w))
    gb = torch.autograd.grad(3 * r2, (h, w))
    for x, y in zip(ga, gb):
        assert torch.allclose(x, y, atol=1e-5)


def test_adam_flat_and_fused_adam_cpu():
    p = torch.randn(100)
    g = torch.randn(100)
    m, v = torch.zeros(100), torch.zeros(100)
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=0.01, weight_decay=0.1)
    for s in (1, 2):
        adam_flat(p, g, m, v, s, 0.01, weight_decay=0.1)
        ref.grad = g.clone()
        opt.step()
    assert torch.allclose(p, ref.detach(), atol=1e-6)
    q = torch.nn.Parameter(torch.randn(10))
    fa = FusedAdam([q], lr=0.1)
    q.grad = torch.ones(10)
    before = q.detach().clone()
    fa.step()
    assert torch.all(q.detach() < before)


def test_grad_clip_cpu():
    ts = [torch.ones(4) * 3, torch.ones(1) * 4]
    s = grad_sumsq(ts)
    assert math.isclose(s.item(), 52.0)
    c = clip_coef(s, 1.0)
    assert abs(c.item() - 1 / math.sqrt(52.0)) < 1e-5


def test_split_column_forward_matches_fused_linear():
    """The odd-N projection forward (two GEMMs into column slices of one output) equals F.linear."""
    import torch.nn.functional as F
    from hcache_deepspeed_amd.runtime.zero.linear import _col_split, _split_fwd
    assert _col_split(6144) == 4096 and _col_split(4096) is None and _col_split(8192) is None
    assert _col_split(4096 + 100) is None and _col_split(14336 * 2) is None
    torch.manual_seed(0)
    x = torch.randn(33, 64)
    w = torch.randn(6144, 64)
    torch.testing.assert_close(_split_fwd(x, w, 4096), F.linear(x, w))


def test_wgrad_pretransposed_and_b2_forms_cpu():
    """ops/gemm.wgrad reference forms on CPU: pre-transposed operands (x2 None -> NT form) and the batched two-half
    split-K path give dY^T X; the b2 heuristic picks only grids that end in a half-empty wave of 256 CUs."""
    from hcache_deepspeed_amd.ops import gemm
    torch.manual_seed(0)
    dy = torch.randn(64, 24)
    x = torch.randn(64, 16)
    ref = dy.t() @ x
    for lay in ("direct", "nt", "direct_b2", "nt_b2"):
        out = torch.zeros(24, 16)
        gemm._wgrad_run(lay, dy, x, out, False)
        torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    out = torch.zeros(24, 16)
    gemm._wgrad_run("nt", dy, None, out, False, dyt=dy.t().contiguous(), xt=x.t().contiguous())
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    out2 = torch.zeros(24, 16)
    gemm.wgrad(dy, None, out2, xt=x.t().contiguous())
    torch.testing.assert_close(out2, ref, rtol=1e-4, atol=1e-4)
    if gemm._B2:
        assert gemm._b2_useful(4096, 14336)       # down: 896 tiles = 3.5 waves
        assert gemm._b2_useful(6144, 4096)        # qkv: 384 tiles = 1.5 waves
        assert not gemm._b2_useful(28672, 4096)   # gate_up: 7 full waves
        assert not gemm._b2_useful(4096, 4096)    # o: 1 full wave
