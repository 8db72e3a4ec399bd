"""Numerics of every HIP kernel against a plain fp32 PyTorch reference of the same op (GPU only)."""
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

from hcache_deepspeed_amd.ops import native  # noqa: E402


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native.load_kernels() is not None, "kernel library must load on the GPU box"
    torch.manual_seed(0)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("H", [4096, 1024, 5120, 2056])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm_fwd_bwd(H, with_res):
    from hcache_deepspeed_amd.ops.norm import rms_norm
    T = 777
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True) if with_res else None
    w = (1 + 0.1 * torch.randn(H, device="cuda", dtype=torch.bfloat16)).requires_grad_(True)
    out = rms_norm(x, w, 1e-5, residual=r)
    y, h = (out if with_res else (out, None))
    # reference
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if with_res else None
    wr = w.detach().float().requires_grad_(True)
    hr = (xr + rr) if with_res else xr
    yr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    assert _rel(y, yr) < 1e-2
    gy = torch.randn_like(y)
    gh = torch.randn_like(y) if with_res else None
    if with_res:
        torch.autograd.backward([y, h], [gy, gh])
        torch.autograd.backward([yr, hr], [gy.float(), gh.float()])
    else:
        y.backward(gy)
        yr.backward(gy.float())
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    if with_res:
        assert _rel(r.grad, rr.grad) < 2e-2


def test_layernorm_fwd_bwd():
    from hcache_deepspeed_amd.ops.norm import layer_norm
    T, H = 513, 768
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = layer_norm(x, w, b, 1e-5)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (H, ), wr, br, 1e-5)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    for a, bb in ((x, xr), (w, wr), (b, br)):
        assert _rel(a.grad, bb.grad) < 2e-2


@pytest.mark.parametrize("interleaved", [False, True])
def test_rope_inplace_and_inverse(interleaved):
    from hcache_deepspeed_amd.ops.rope import rope_, rope_tables
    T, nh, D = 300, 12, 128
    S = 100
    cos, sin = rope_tables(4096, D, 500000.0, device="cuda")
    x = torch.randn(T, nh + 4, D, device="cuda", dtype=torch.bfloat16)
    ref = x.clone()
    rope_(x, cos, sin, nh, seq_len=S, interleaved=interleaved)
    # torch reference
    pos = torch.arange(T, device="cuda") % S
    c, s = cos[pos][:, None], sin[pos][:, None]
    xf = ref[:, :nh].float()
    if not interleaved:
        a, b = xf[..., :D // 2], xf[..., D // 2:]
        exp = torch.cat([a * c - b * s, b * c + a * s], -1)
    else:
        a, b = xf[..., 0::2], xf[..., 1::2]
        exp = torch.stack([a * c - b * s, b * c + a * s], -1).flatten(-2)
    assert _rel(x[:, :nh], exp) < 1e-2
    assert torch.equal(x[:, nh:], ref[:, nh:])
    rope_(x, cos, sin, nh, seq_len=S, sign=-1.0, interleaved=interleaved)
    assert _rel(x, ref) < 2e-2


@pytest.mark.parametrize("T,I", [(333, 1024), (7, 8), (3, 24), (130, 2056)])
@pytest.mark.parametrize("act", ["silu", "gelu_tanh", "relu"])
def test_glu(act, T, I):
    from hcache_deepspeed_amd.ops.activations import glu, _ref_act, act_code
    gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = glu(gu, act)
    gr = gu.detach().float().requires_grad_(True)
    g, u = gr.split(I, -1)
    yr = _ref_act(g, act_code(act)) * u
    assert _rel(y, yr) < 1e-2
    d = torch.randn_like(y)
    y.backward(d)
    yr.backward(d.float())
    assert _rel(gu.grad, gr.grad) < 2e-2


def test_adam_flat_matches_torch():
    from hcache_deepspeed_amd.ops.optimizers import adam_flat
    n = 1_000_003
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    lp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    ref = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        adam_flat(p, g, m, v, step, 1e-3, (0.9, 0.95), 1e-8, 0.1, adamw=True, lp_out=lp, grad_scale=0.5)
        ref.grad = g.float() * 0.5
        opt.step()
    assert (p - ref.detach()).abs().max().item() < 1e-5
    assert torch.equal(lp, p.to(torch.bfloat16))


def test_fused_adam_multi_tensor():
    from hcache_deepspeed_amd.ops.optimizers import FusedAdam
    shapes = [(1000, 37), (4096, ), (3, 5, 7), (70001, )]
    ps = [torch.randn(s, device="cuda", requires_grad=True) for s in shapes]
    rs = [p.detach().clone().requires_grad_(True) for p in ps]
    opt = FusedAdam(ps, lr=1e-2, weight_decay=0.01)
    ropt = torch.optim.AdamW(rs, lr=1e-2, weight_decay=0.01)
    for _ in range(3):
        for p, r in zip(ps, rs):
            g = torch.randn_like(p)
            p.grad, r.grad = g, g.clone()
        opt.step()
        ropt.step()
    for p, r in zip(ps, rs):
        assert (p - r).abs().max().item() < 1e-5


def test_lion_and_lamb_run():
    from hcache_deepspeed_amd.ops.optimizers import FusedLamb, FusedLion
    for cls in (FusedLion, FusedLamb):
        p = torch.randn(10000, device="cuda", requires_grad=True)
        ref = p.detach().cpu().clone().requires_grad_(True)
        opt, ropt = cls([p], lr=1e-3), cls([ref], lr=1e-3)
        g = torch.randn(10000)
        p.grad, ref.grad = g.cuda(), g.clone()
        opt.step()
        ropt.step()
        assert (p.detach().cpu() - ref.detach()).abs().max().item() < 1e-5


def test_grad_norm_and_clip():
    from hcache_deepspeed_amd.ops.optimizers import clip_coef, grad_sumsq
    ts = [torch.randn(12345, device="cuda", dtype=torch.bfloat16), torch.randn(999, device="cuda")]
    fi = torch.zeros(1, device="cuda", dtype=torch.int32)
    s = grad_sumsq(ts, found_inf=fi)
    exp = sum((t.float()**2).sum() for t in ts)
    assert abs(s.item() - exp.item()) / exp.item() < 1e-4
    assert fi.item() == 0
    c = clip_coef(s, 1.0)
    assert abs(c.item() - min(1.0, 1.0 / (math.sqrt(exp.item()) + 1e-6))) < 1e-4
    ts[0][7] = float("inf")
    grad_sumsq(ts, found_inf=fi)
    assert fi.item() == 1


@pytest.mark.parametrize("V", [128256, 50257, 1000])
def test_cross_entropy(V):
    from hcache_deepspeed_amd.ops.cross_entropy import cross_entropy
    T = 257
    logits = (3 * torch.randn(T, V, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, V, (T, ), device="cuda")
    tgt[::7] = -100
    loss = cross_entropy(logits, tgt)
    lr = logits.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr, tgt, ignore_index=-100)
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1, abs(ref.item()))
    loss.backward()
    ref.backward()
    assert _rel(logits.grad, lr.grad) < 2e-2


def test_fused_linear_cross_entropy():
    from hcache_deepspeed_amd.ops.cross_entropy import fused_linear_cross_entropy
    T, H, V = 1000, 256, 5003
    h = (0.5 * torch.randn(T, H, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    w = (0.05 * torch.randn(V, H, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    t = torch.randint(0, V, (T, ), device="cuda")
    t[:10] = -100
    loss = fused_linear_cross_entropy(h, w, t, chunk_rows=384)
    hr, wr = h.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(hr @ wr.t(), t)
    assert abs(loss.item() - ref.item()) < 2e-3 * abs(ref.item())
    (2 * loss).backward()
    (2 * ref).backward()
    assert _rel(h.grad, hr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2
    from hcache_deepspeed_amd.ops import cross_entropy as C
    assert C._ADDMM_OUT_DTYPE[0] is True, "fused fp32-accumulating LM-head GEMM silently disabled"


def _attn_ref(q, k, v, causal, window=0, cu=None, S=None):
    from hcache_deepspeed_amd.ops.attention import _ref_attention_f32
    scale = 1 / math.sqrt(q.shape[-1])
    o, _ = _ref_attention_f32(q, k, v, causal, scale, cu, S, window)
    return o


@pytest.mark.parametrize("S,Hq,Hkv,causal,window", [(256, 4, 2, True, 0), (1000, 8, 2, True, 0),
                                                     (384, 4, 4, False, 0), (700, 4, 1, True, 129),
                                                     (64, 2, 1, True, 0), (2048, 8, 8, True, 0)])
def test_flash_attn_fwd_bwd(S, Hq, Hkv, causal, window):
    from hcache_deepspeed_amd.ops.attention import flash_attn
    B, D = 2, 128
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn(q, k, v, causal=causal, window=window)
    qr, kr, vr = (t.detach().float().reshape(B * S, t.shape[2], D).requires_grad_(True) for t in (q, k, v))
    orf = _attn_ref(qr, kr, vr, causal, window, None, S)
    assert _rel(o.reshape(B * S, Hq, D), orf) < 1e-2
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float().reshape(B * S, Hq, D))
    assert _rel(q.grad.reshape(B * S, Hq, D), qr.grad) < 2e-2
    assert _rel(k.grad.reshape(B * S, Hkv, D), kr.grad) < 2e-2
    assert _rel(v.grad.reshape(B * S, Hkv, D), vr.grad) < 2e-2


@pytest.fixture
def no_attn_fallback(monkeypatch):
    """Fail the test if the fp32 torch reference attention runs instead of the HIP kernels."""
    from hcache_deepspeed_amd.ops import attention as A

    def boom(*a, **k):
        raise AssertionError("torch reference attention ran on the GPU path")

    monkeypatch.setattr(A, "_ref_attention", boom)
    monkeypatch.setattr(A, "_padded_ref", boom)
    monkeypatch.setattr(A, "_ref_bwd", boom)


@pytest.mark.parametrize("D", [32, 48, 64, 80, 96, 112, 160, 192, 256])
@pytest.mark.parametrize("causal,window", [(True, 0), (False, 0), (True, 97)])
def test_flash_attn_head_dims(D, causal, window, no_attn_fallback):
    """Every instantiated head dim (GPT-2/BERT/Falcon/OPT 64, Phi 80, Phi-3 96, Gemma 256, ...) on the HIP path
    against the fp32 reference, forward and backward, GQA, ragged tile edges."""
    from hcache_deepspeed_amd.ops.attention import flash_attn
    B, S, Hq, Hkv = 2, 333, 4, 2
    torch.manual_seed(D)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn(q, k, v, causal=causal, window=window)
    qr, kr, vr = (t.detach().float().reshape(B * S, t.shape[2], D).requires_grad_(True) for t in (q, k, v))
    orf = _attn_ref(qr, kr, vr, causal, window, None, S)
    assert _rel(o.reshape(B * S, Hq, D), orf) < 1e-2
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float().reshape(B * S, Hq, D))
    assert _rel(q.grad.reshape(B * S, Hq, D), qr.grad) < 2e-2
    assert _rel(k.grad.reshape(B * S, Hkv, D), kr.grad) < 2e-2
    assert _rel(v.grad.reshape(B * S, Hkv, D), vr.grad) < 2e-2


@pytest.mark.parametrize("D", [64, 128])
def test_flash_attn_padding_seq_lens(D, no_attn_fallback):
    """Right-padded batch + key-padding lengths (the BERT mask case) on the HIP kernels: valid rows match the
    per-sequence reference, padded rows and their gradients are zero."""
    from hcache_deepspeed_amd.ops.attention import flash_attn
    B, S, H = 3, 200, 4
    lens = torch.tensor([200, 77, 1], dtype=torch.int32)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn(q, k, v, causal=False, seq_lens=lens.cuda())
    do = torch.randn_like(o)
    o.backward(do)
    for b, L in enumerate(lens.tolist()):
        qr, kr, vr = (t.detach()[b, :L].float().requires_grad_(True) for t in (q, k, v))
        orf = _attn_ref(qr, kr, vr, False, 0, None, L)
        assert _rel(o[b, :L], orf) < 1e-2
        orf.backward(do[b, :L].float())
        for got, want in ((q.grad[b, :L], qr.grad), (k.grad[b, :L], kr.grad), (v.grad[b, :L], vr.grad)):
            # L == 1: softmax is exactly 1, so dq / dk are 0 up to rounding -- compare absolutely there
            err = (got.float() - want).norm().item()
            assert err < 2e-2 * want.norm().item() + 1e-4 * math.sqrt(want.numel())
        assert o[b, L:].abs().max().item() == 0 if L < S else True
        assert k.grad[b, L:].abs().max().item() == 0 if L < S else True


def test_flash_attn_varlen():
    from hcache_deepspeed_amd.ops.attention import flash_attn
    lens = [17, 300, 1, 129, 64]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), device="cuda", dtype=torch.int32)
    T, Hq, Hkv, D = sum(lens), 4, 2, 128
    q = torch.randn(T, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(T, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(T, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = flash_attn(q, k, v, causal=True, cu_seqlens=cu)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = _attn_ref(qr, kr, vr, True, 0, cu.cpu(), None)
    assert _rel(o, orf) < 1e-2
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    for a, b in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, b.grad) < 2e-2


def test_flash_attn_lse_spike():
    """Force the online-softmax rescale: one key row far larger than the rest (guide §5.4 rule 26)."""
    from hcache_deepspeed_amd.ops.attention import flash_attn
    B, S, H, D = 1, 512, 2, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k[:, 300] = q[:, 400] * 4  # spike at tile 4 for query 400
    o, lse = flash_attn(q, k, v, causal=True, return_lse=True)
    orf = _attn_ref(*(t.float().reshape(S, H, D) for t in (q, k, v)), True, 0, None, S)
    assert _rel(o.reshape(S, H, D), orf) < 1e-2


def test_qkv_attention_matches_unfused():
    from hcache_deepspeed_amd.ops.attention import qkv_attention, flash_attn
    from hcache_deepspeed_amd.ops.rope import apply_rotary, rope_tables
    B, S, Hq, Hkv, D = 2, 512, 8, 2, 128
    T = B * S
    cos, sin = rope_tables(S, D, 500000.0, device="cuda")
    qkv = torch.randn(T, Hq + 2 * Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    x1 = qkv.detach().clone().requires_grad_(True)
    o1 = qkv_attention(qkv.clone(), Hq, Hkv, cos, sin, seq_len=S)
    q = apply_rotary(x1[:, :Hq], cos, sin, seq_len=S)
    k = apply_rotary(x1[:, Hq:Hq + Hkv], cos, sin, seq_len=S)
    v = x1[:, Hq + Hkv:].contiguous()
    o2 = flash_attn(q.view(B, S, Hq, D), k.view(B, S, Hkv, D), v.view(B, S, Hkv, D)).reshape(T, Hq * D)
    assert _rel(o1, o2) < 1e-2
    g = torch.randn_like(o1)
    o1.backward(g)
    o2.backward(g)
    assert _rel(qkv.grad, x1.grad) < 2e-2


def _paged_setup(lens, seen, Hq=8, Hkv=2, D=128, bs=64, nblocks=64, rot=None):
    from hcache_deepspeed_amd.ops.rope import rope_tables
    torch.manual_seed(3)
    cache = torch.randn(nblocks, bs, 2, Hkv, D, device="cuda", dtype=torch.bfloat16)
    perm = torch.randperm(nblocks).tolist()
    tables, metas, off = [], [], 0
    maxb = 0
    for n, s in zip(lens, seen):
        nb = (n + s + bs - 1) // bs
        tables.append([perm.pop() for _ in range(nb)])
        maxb = max(maxb, nb)
        metas.append((off, n, s))
        off += n
    tab = torch.zeros(len(lens), maxb, dtype=torch.int32)
    for i, t in enumerate(tables):
        tab[i, :len(t)] = torch.tensor(t)
    return cache, tab, metas, off, rope_tables(4096, rot or D, 10000.0, device="cuda")


@pytest.mark.parametrize("D,rot", [(128, 0), (64, 0), (80, 32), (80, 40), (96, 0), (256, 64)])
def test_kv_rope_scatter_matches_reference(D, rot):
    """Fused RoPE + paged KV scatter for every serving head dim, incl. partial rotary (Phi: 80 / 32)."""
    from hcache_deepspeed_amd.ops.paged import kv_rope_scatter
    lens, seen = [5, 70, 1], [0, 10, 200]
    Hq, Hkv = 8, 2
    cache, tab, metas, T, (cos, sin) = _paged_setup(lens, seen, D=D, rot=rot)
    tok_seq = torch.cat([torch.full((n, ), i, dtype=torch.int32) for i, n in enumerate(lens)])
    tok_pos = torch.cat([torch.arange(s, s + n, dtype=torch.int32) for n, s in zip(lens, seen)])
    qkv = torch.randn(T, Hq + 2 * Hkv, D, device="cuda", dtype=torch.bfloat16)
    q2, c2 = qkv.clone().cpu().float(), cache.clone().cpu().float()
    kv_rope_scatter(qkv, cache, tok_seq.cuda(), tok_pos.cuda(), tab.cuda(), cos, sin, Hq, Hkv, rotary_dim=rot)
    kv_rope_scatter(q2, c2, tok_seq, tok_pos, tab, cos.cpu(), sin.cpu(), Hq, Hkv, rotary_dim=rot)
    assert _rel(qkv.cpu(), q2) < 1e-2
    assert _rel(cache.cpu(), c2) < 1e-2


@pytest.mark.parametrize("D", [128, 64, 80, 96, 256])
@pytest.mark.parametrize("lens,seen", [([1, 1, 1], [100, 5, 700]), ([130, 64, 3], [0, 0, 0]), ([37, 1], [90, 333])])
def test_paged_attention_matches_reference(lens, seen, D):
    from hcache_deepspeed_amd.ops.paged import build_atoms, paged_attention
    Hq, Hkv = 8, 2
    cache, tab, metas, T, _ = _paged_setup(lens, seen, D=D)
    q = torch.randn(T, Hq, D, device="cuda", dtype=torch.bfloat16)
    atoms, n = build_atoms(metas, Hq, Hkv)
    meta = torch.tensor(metas, dtype=torch.int32)
    o = paged_attention(q, cache, atoms.cuda(), n, meta.cuda(), tab.cuda(), Hq, Hkv, 1 / math.sqrt(D))
    ref = paged_attention(q.cpu().float(), cache.cpu().float(), atoms, n, meta, tab, Hq, Hkv, 1 / math.sqrt(D),
                          seq_meta_host=metas, block_tables_host=tab)
    assert _rel(o.cpu(), ref) < 1e-2


@pytest.mark.parametrize("D,G", [(128, 4), (64, 8), (256, 2), (128, 1)])
@pytest.mark.parametrize("seen,window", [([100, 5, 700, 0], 0), ([1000, 33, 64, 63], 0), ([300, 2000, 7, 90], 50)])
@pytest.mark.parametrize("merge", [False, True])
def test_paged_decode_matches_reference(seen, window, D, G, merge, monkeypatch):
    """Split-K paged decode (one new token per sequence) against the torch reference over the same block tables,
    incl. sliding window, a first-token sequence (seen 0) and splits that get no keys; ``merge``: the last workgroup
    of each (sequence, kv head) merges the splits in the same launch (its counters must be back at zero after)."""
    from hcache_deepspeed_amd.ops import paged as P
    from hcache_deepspeed_amd.ops.paged import build_atoms, paged_attention
    monkeypatch.setattr(P, "_MERGE_IN_KERNEL", merge)
    Hkv = 2
    Hq = Hkv * G
    lens = [1] * len(seen)
    cache, tab, metas, T, _ = _paged_setup(lens, seen, D=D)
    q = torch.randn(T, Hq, D, device="cuda", dtype=torch.bfloat16)
    atoms, n = build_atoms(metas, Hq, Hkv)
    meta = torch.tensor(metas, dtype=torch.int32)
    o = paged_attention(q, cache, atoms.cuda(), n, meta.cuda(), tab.cuda(), Hq, Hkv, 1 / math.sqrt(D), window,
                        decode=True)
    o_atom = paged_attention(q, cache, atoms.cuda(), n, meta.cuda(), tab.cuda(), Hq, Hkv, 1 / math.sqrt(D), window)
    ref = paged_attention(q.cpu().float(), cache.cpu().float(), atoms, n, meta, tab, Hq, Hkv, 1 / math.sqrt(D), window,
                          seq_meta_host=metas, block_tables_host=tab)
    assert _rel(o.cpu(), ref) < 1e-2
    assert _rel(o.cpu(), o_atom.cpu()) < 1e-2
    if merge:
        for _ in range(3):  # repeated launches reuse the counters: each must find them zeroed again
            o2 = paged_attention(q, cache, atoms.cuda(), n, meta.cuda(), tab.cuda(), Hq, Hkv, 1 / math.sqrt(D), window,
                                 decode=True)
            assert torch.equal(o2, o)
        assert int(P._COUNTERS[q.device].abs().sum()) == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_moe_dispatch_combine_fwd_bwd(dtype):
    from hcache_deepspeed_amd.ops import moe as M
    T, H, E, k = 1000, 1024, 8, 2
    x = torch.randn(T, H, device="cuda", dtype=dtype, requires_grad=True)
    logits = torch.randn(T, E, device="cuda")
    expert, pos, w, C, _, _ = M.topk_route(logits, k, capacity_factor=1.0, min_capacity=4)
    assert (pos >= C).any()  # some drops at capacity factor 1.0
    w = w.requires_grad_(True)
    d = M.moe_dispatch(x, expert, pos, E, C)
    y = (d.float() * 1.5 + 0.25).to(dtype)  # stand-in expert
    out = M.moe_combine(y, expert, pos, w, C)
    g = torch.randn_like(out)
    (out.float() * g.float()).sum().backward()
    # fp32 reference through the torch reference paths
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    dr = M._ref_dispatch(xr, expert, pos, E, C)
    yr = dr * 1.5 + 0.25
    outr = M._ref_combine(yr, expert, pos, wr, C)
    (outr * g.float()).sum().backward()
    assert torch.equal(d.float(), M._ref_dispatch(x.detach().float(), expert, pos, E, C).to(dtype).float())
    assert _rel(out, outr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-2


def test_mixtral_tiny_train_step_gpu():
    from hcache_deepspeed_amd.models.mixtral import MixtralForCausalLM, tiny_moe
    torch.manual_seed(0)
    m = MixtralForCausalLM(tiny_moe()).cuda().to(torch.bfloat16)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    x = torch.randint(0, 512, (2, 256), device="cuda")
    losses = []
    for _ in range(5):
        loss = m(x, labels=x)
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
    assert all(math.isfinite(v) for v in losses) and losses[-1] < losses[0]


@pytest.mark.parametrize("bits,sym", [(8, True), (8, False), (4, True), (4, False)])
def test_quant_int_matches_reference(bits, sym):
    from hcache_deepspeed_amd.ops import quantizer as Q
    x = torch.randn(64 * 2048, device="cuda", dtype=torch.bfloat16)
    q, s, m = Q.quantize(x, 2048, bits, sym)
    qr, sr, mr = Q._ref_quant_int(x.cpu(), 2048, bits, sym)
    assert torch.allclose(s.cpu(), sr, rtol=1e-6)
    # rounding ties may differ in the last unit on a handful of elements
    y = Q.dequantize(q, s, m, 2048, bits, sym, torch.float32)
    yr = Q._ref_dequant_int(qr, sr, mr, 2048, bits, sym, torch.float32)
    assert (y.cpu() - yr).abs().max() <= s.max().item() * 1.01
    assert (y.cpu() - x.float().cpu()).abs().max() <= s.max().item() * 0.51


@pytest.mark.parametrize("fmt", ["e4m3", "e5m2"])
def test_quant_fp8_matches_torch_ocp(fmt):
    from hcache_deepspeed_amd.ops import quantizer as Q
    x = torch.randn(32 * 512, device="cuda", dtype=torch.float32) * 3
    q, s = Q.quantize_fp8(x, 512, fmt)
    qr, sr = Q.quantize_fp8(x.cpu(), 512, fmt)
    assert torch.allclose(s.cpu(), sr)
    # gfx950 converts to the OCP formats: bit-exact with torch's float8 casts (RNE)
    mism = (q.cpu() != qr).float().mean().item()
    assert mism < 1e-3, mism
    y = Q.dequantize_fp8(q, s, 512, fmt, torch.float32)
    assert torch.allclose(y.cpu(), Q.dequantize_fp8(qr, sr, 512, fmt, torch.float32), rtol=0.07, atol=1e-6)


@pytest.mark.parametrize("bits", [8, 4])
def test_dequant_reduce(bits):
    from hcache_deepspeed_amd.ops import quantizer as Q
    W, n = 4, 8192
    xs = [torch.randn(n, device="cuda", dtype=torch.bfloat16) for _ in range(W)]
    qs = [Q.quantize(x, 512, bits, True) for x in xs]
    q = torch.cat([a[0] for a in qs])
    s = torch.cat([a[1] for a in qs])
    out = Q.dequant_reduce(q, s, W, n, 512, bits)
    ref = Q.dequant_reduce(q.cpu(), s.cpu(), W, n, 512, bits)
    assert torch.allclose(out.cpu(), ref, atol=1e-5, rtol=1e-5)
    acc = torch.ones(n, device="cuda")
    Q.dequant_reduce(q, s, W, n, 512, bits, out=acc, accumulate=True)
    assert torch.allclose(acc.cpu(), ref + 1, atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("pad", [None, 3])
def test_embedding_grad_scatter_add_gpu(dtype, pad):
    from hcache_deepspeed_amd.ops.embedding import embedding_grad_add_
    torch.manual_seed(0)
    V, D, N = 1000, 4096 + 8 * 3, 5000
    ids = torch.randint(0, V, (N, ), device="cuda")
    ids[:600] = 7  # a long run of one id
    ids[600:700] = 3
    dy = torch.randn(N, D, device="cuda", dtype=dtype)
    grad = torch.randn(V, D, device="cuda", dtype=dtype)
    ref = grad.float().clone()
    keep = ids != (pad if pad is not None else -1)
    ref.index_add_(0, ids[keep], dy[keep].float())
    out = embedding_grad_add_(grad, ids, dy, pad)
    assert out.data_ptr() == grad.data_ptr()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(grad.float(), ref, atol=tol * 8, rtol=tol)
    again = torch.randn(V, D, device="cuda", dtype=dtype)
    a2 = again.clone()
    embedding_grad_add_(again, ids, dy, pad)
    embedding_grad_add_(a2, ids, dy, pad)
    assert torch.equal(again, a2)  # deterministic


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 384), (1280, 512, 1024), (2304, 2560, 256)])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("variant", [0, 1])
def test_gemm_nt_matches_fp32_gpu(M, N, K, accumulate, variant):
    from hcache_deepspeed_amd.ops import native
    from hcache_deepspeed_amd.ops.gemm import gemm_nt
    assert native.kernels().hds_gemm_nt_supported(M, N, K, K, K, N)
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    # asymmetric structure: a row/column pattern that a transposed or mis-indexed store cannot reproduce
    a[:, 0] = torch.arange(M, device="cuda", dtype=torch.float32).to(torch.bfloat16) / M
    b[:, 1] = torch.arange(N, device="cuda", dtype=torch.float32).to(torch.bfloat16) / N
    c0 = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    out = c0.clone()
    gemm_nt(a, b, out=out, alpha=0.5, accumulate=accumulate, variant=variant)
    ref = 0.5 * (a.float() @ b.float().t()) + (c0.float() if accumulate else 0)
    err = (out.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err


@pytest.mark.gpu
def test_mx_quantize_matches_reference_gpu():
    from hcache_deepspeed_amd.ops.fp8_gemm import mx_quantize, mx_quantize_ref
    torch.manual_seed(0)
    x = (torch.randn(512, 1024, device="cuda") * torch.logspace(-3, 3, 1024, device="cuda")).to(torch.bfloat16)
    x[3, :32] = 0  # all-zero block
    q, s = mx_quantize(x)
    qr, sr = mx_quantize_ref(x.cpu())
    assert torch.equal(s.cpu(), sr)
    mism = (q.cpu() != qr).float().mean().item()
    assert mism < 1e-3, mism  # rounding ties may differ in the last bit only


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (512, 768, 512), (1280, 512, 2048)])
@pytest.mark.parametrize("variant", [0, 1])
def test_mx_gemm_matches_dequant_reference_gpu(M, N, K, variant):
    from hcache_deepspeed_amd.ops.fp8_gemm import mx_dequantize, mx_gemm, mx_quantize
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    a[:, :128] *= 50  # blocks with very different scales along K
    b[:, 256:] *= 1e-2 if K > 256 else 1
    a[:, 0] = torch.arange(M, device="cuda", dtype=torch.float32).to(torch.bfloat16) / M
    qa, sa = mx_quantize(a)
    qb, sb = mx_quantize(b)
    out = mx_gemm(qa, sa, qb, sb, alpha=0.5, variant=variant)
    ref = 0.5 * (mx_dequantize(qa, sa) @ mx_dequantize(qb, sb).t())
    err = (out.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    # and the quantized product tracks the bf16 one
    full = 0.5 * (a.float() @ b.float().t())
    rel = ((out.float() - full).norm() / full.norm()).item()
    assert rel < 0.08, rel


@pytest.mark.gpu
def test_quantized_lora_linear_mx_fp8_gpu():
    """LoRA over an MX-FP8 frozen base: forward and input gradient on the FP8 matrix cores match the
    dequantized-weight computation."""
    from hcache_deepspeed_amd.linear import LoRAConfig, OptimizedLinear, QuantizationConfig
    from hcache_deepspeed_amd.ops.fp8_gemm import mx_dequantize, mx_quantize
    torch.manual_seed(0)
    lin = OptimizedLinear(1024, 512, lora_config=LoRAConfig(lora_r=8, lora_alpha=16),
                          quantization_config=QuantizationConfig(q_bits=8, group_size=256, mx_fp8=True),
                          dtype=torch.bfloat16, device="cuda")
    lin.weight.to("cuda")
    assert lin.weight.mx_ok()
    x = torch.randn(2, 256, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = lin(x)
    w = mx_dequantize(*lin.weight.mx_w)
    xq = mx_dequantize(*mx_quantize(x.detach().reshape(-1, 1024)))
    ref = (xq @ w.t()).reshape(2, 256, 512)
    base = y - lin.lora_scaling_factor * lin.lora_weight_2(lin.lora_weight_1(x))
    err = (base.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err
    g = torch.randn_like(y)
    y.backward(g)
    dx_ref = g.float().reshape(-1, 512) @ w + lin.lora_scaling_factor * (
        g.float().reshape(-1, 512) @ lin.lora_weight_2.weight.float() @ lin.lora_weight_1.weight.float())
    rel = ((x.grad.float().reshape(-1, 1024) - dx_ref).norm() / dx_ref.norm()).item()
    assert rel < 0.08, rel
    assert lin.lora_weight_1.weight.grad is not None


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 128, 256])
@pytest.mark.parametrize("H,Hkv", [(8, 8), (32, 8), (16, 2)])
@pytest.mark.parametrize("S", [1, 37, 700, 5000])
def test_decode_attention_matches_reference_gpu(D, H, Hkv, S):
    from hcache_deepspeed_amd.ops.decode_attention import decode_attention, decode_attention_ref, decode_supported
    torch.manual_seed(S + D)
    B = 3
    qf = torch.randn(B, H, 1, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16)
    q = qf[:, :, 0]  # strided view, as the attention interface passes it
    assert decode_supported(q, k)
    bias = torch.zeros(B, S, device="cuda")
    bias[1, :S // 3] = float("-inf")  # left padding of one sequence
    alibi = torch.linspace(0.01, 0.5, H, device="cuda")
    for kw in ({}, {"bias": bias}, {"alibi": alibi}, {"bias": bias, "alibi": alibi}):
        if S == 1 and "bias" in kw:
            continue
        out = decode_attention(q, k, v, 0.1, **kw)
        ref = decode_attention_ref(q.float(), k.float(), v.float(), 0.1, kw.get("bias"), kw.get("alibi"))
        torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)
    # device lengths + sliding window: masked lanes at split tails, before the window and past lens[b]; the
    # cache past lens is filled with NaN so a masked lane that reads or accumulates it poisons the output
    if S >= 37:
        lens = torch.tensor([S, max(1, S // 2), max(1, S - 5)], device="cuda", dtype=torch.int32)
        kn, vn = k.clone(), v.clone()
        for b, n in enumerate(lens.tolist()):
            kn[b, :, n:] = float("nan")
            vn[b, :, n:] = float("nan")
        for win in (0, 17):
            out = decode_attention(q, kn, vn, 0.1, lens=lens, window=win)
            assert torch.isfinite(out.float()).all()
            for b, n in enumerate(lens.tolist()):
                lo = max(0, n - win) if win else 0
                ref = decode_attention_ref(q[b:b + 1].float(), k[b:b + 1, :, lo:n].float(), v[b:b + 1, :, lo:n].float(),
                                           0.1)
                torch.testing.assert_close(out[b:b + 1].float(), ref.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [5, 20])
@pytest.mark.parametrize("case", ["causal", "full", "window", "varlen"])
def test_flash_fwd_staggered_variant_gpu(case, variant):
    """The shipped forward variants 5 (8-wave software-pipelined softmax, the fallback) and 20 (one wave per SIMD, the
    default) against variant 2 and the fp32 reference; the backward (which consumes the forward's LSE) must agree too.
    The shipped library refuses every other variant (experiments and wrong-result diagnostics live in the A/B
    library only)."""
    from hcache_deepspeed_amd.ops import native
    from hcache_deepspeed_amd.ops.attention import flash_attn
    lib = native.kernels()
    torch.manual_seed(7)
    B, S, Hq, Hkv, D = 2, 700, 8, 2, 128
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    kw = dict(causal=case != "full", window=100 if case == "window" else 0)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    assert lib.hds_attn_diag_build() == 0
    for bad in (4, 9, 11, 12, 13, 14, 15, 16, 17, 18, 19, 21, 22):
        assert lib.hds_attn_fwd_variant(bad) != 0, bad
    try:
        outs, grads = {}, {}
        for var in (2, variant):
            assert lib.hds_attn_fwd_variant(var) == 0
            qg, kg, vg = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
            if case == "varlen":
                cu = torch.tensor([0, 333, 2 * S], device="cuda", dtype=torch.int32)
                o = flash_attn(qg.reshape(-1, Hq, D), kg.reshape(-1, Hkv, D), vg.reshape(-1, Hkv, D),
                               causal=True, cu_seqlens=cu).reshape(B, S, Hq, D)
            else:
                o = flash_attn(qg, kg, vg, **kw)
            o.backward(do)
            outs[var] = o.detach()
            grads[var] = (qg.grad, kg.grad, vg.grad)
    finally:
        lib.hds_attn_fwd_variant(native.fwd_variant_default())  # the library default
    d = (outs[variant].float() - outs[2].float()).abs().max().item()
    assert d < 3e-2, d  # both within bf16 rounding of each other (same math, different schedule)
    for a, b in zip(grads[variant], grads[2]):
        rel = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert rel < 2e-2, rel
    outs[4] = outs[variant]
    if case != "varlen":
        qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k.repeat_interleave(4, 2), v.repeat_interleave(4, 2)))
        s = qf @ kf.transpose(-1, -2) / D**0.5
        i = torch.arange(S, device="cuda")
        mask = torch.zeros(S, S, dtype=torch.bool, device="cuda")
        if kw["causal"]:
            mask |= i[None, :] > i[:, None]
        if kw["window"]:
            mask |= i[None, :] <= i[:, None] - kw["window"]
        ref = (torch.softmax(s.masked_fill(mask, float("-inf")), -1) @ vf).transpose(1, 2)
        torch.testing.assert_close(outs[4].float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("window", [0, 40])
def test_hip_graph_decode_matches_eager_gpu(window, monkeypatch):
    """KV-cached greedy generation with the decode step captured in a HIP graph (device-side positions / cache slot /
    lengths, decode_attention(lens=...)) produces exactly the tokens of the eager loop, incl. left padding."""
    from hcache_deepspeed_amd.models.generation import KVCacheGenerator
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(hidden_size=512, intermediate_size=1024, num_hidden_layers=3, num_attention_heads=4,
                              num_key_value_heads=2, vocab_size=1000, sliding_window=window)).cuda().to(
                                  torch.bfloat16).eval()
    g = torch.Generator(device="cuda").manual_seed(1)
    prompt = torch.randint(1, 1000, (3, 50), device="cuda", generator=g)
    mask = torch.ones_like(prompt)
    mask[1, :7] = 0
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("HDS_DECODE_GRAPH", mode)
        gen = KVCacheGenerator(m)
        outs[mode] = gen.generate(prompt, attention_mask=mask, max_new_tokens=24)
        assert gen.used_graph == (mode == "1")
    assert torch.equal(outs["1"], outs["0"])


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 6144, 4096), (3, 4100, 4096), (8, 1000, 1032), (5, 128256, 512), (2, 7, 8)])
def test_gemv_bf16_matches_fp32(M, N, K):
    """Decode-sized HIP GEMV (ops/gemv.py) against an fp32 reference, incl. odd N (row tail), K not a multiple of
    the 1024-element double chunk, bias, and a strided activation view."""
    from hcache_deepspeed_amd.ops.gemv import gemv, gemv_ok
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    w = (torch.randn(N, K, device="cuda", generator=g) * K**-0.5).to(torch.bfloat16)
    big = torch.randn(M, K + 8, device="cuda", generator=g).to(torch.bfloat16)
    x = big[:, :K]  # row stride K + 8
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    assert gemv_ok(x, w, b) or N * K > __import__("hcache_deepspeed_amd.ops.gemv", fromlist=["x"]).max_numel(M)
    y = gemv(x, w, b)
    ref = x.float() @ w.float().t() + b.float()
    rel = ((y.float() - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(2, 6144, 4096), (8, 28672, 4096), (16, 4096, 14336), (5, 1000, 1024),
                                   (3, 7, 128)])
def test_skinny_gemm_matches_fp32(M, N, K):
    """The matrix-core skinny GEMM (2..16 token rows) against an fp32 reference, incl. an N tail, bias and a strided
    activation view; the HIP path must be the one that ran."""
    from hcache_deepspeed_amd.ops.gemv import linear, skinny, skinny_ok
    g = torch.Generator(device="cuda").manual_seed(M * 13 + N)
    w = (torch.randn(N, K, device="cuda", generator=g) * K**-0.5).to(torch.bfloat16)
    big = torch.randn(M, K + 8, device="cuda", generator=g).to(torch.bfloat16)
    x = big[:, :K]  # row stride K + 8
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    assert skinny_ok(x, w, b)
    ref = x.float() @ w.float().t() + b.float()
    for y in (skinny(x, w, b), linear(x, w, b)):
        rel = ((y.float() - ref).norm() / ref.norm()).item()
        assert rel < 8e-3, rel


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,glu,res", [(1, 6144, 4096, False, True), (1, 14336, 4096, True, True),
                                           (3, 4100, 4096, False, False), (8, 1000, 1032, True, True),
                                           (5, 8192, 512, True, False)])
def test_gemv_fused_norm_glu_matches_fp32(M, N, K, glu, res):
    """The decode GEMV with the RMSNorm prologue (and the SwiGLU epilogue) against fp32 references of the same
    arithmetic: the new residual is bit-exact (one bf16 add), the normed rows within a bf16 ulp, the outputs at
    GEMV accuracy; the HIP path must be the one that ran."""
    from hcache_deepspeed_amd.ops import gemv as G
    g = torch.Generator(device="cuda").manual_seed(M * 11 + N)
    rows = 2 * N if glu else N
    w = (torch.randn(rows, K, device="cuda", generator=g) * K**-0.5).to(torch.bfloat16)
    h = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    r0 = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16) if res else None
    gamma = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    assert G.fused_ok(h, w, gamma, glu)
    y, r, x = G.fused_gemv(h, w, r0, gamma, 1e-5, glu=glu, want_x=True)
    rr = h if r0 is None else (h.float() + r0.float()).to(torch.bfloat16)
    assert torch.equal(r, rr)
    rf = rr.float()
    xr = rf * torch.rsqrt(rf.square().mean(-1, keepdim=True) + 1e-5) * gamma.float()
    assert ((x.float() - xr).abs() <= 1e-2 * xr.abs() + 1e-3).all()
    yr = x.float() @ w.float().t()
    if glu:
        yr = torch.nn.functional.silu(yr[:, :N].to(torch.bfloat16).float()) * yr[:, N:].to(torch.bfloat16).float()
    rel = ((y.float() - yr).norm() / yr.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.gpu
def test_kv_append_matches_index_copy():
    """HIP KV append (slot read on the device) equals two index_copy_ calls, for strided K/V views of a fused qkv."""
    from hcache_deepspeed_amd.ops.decode_attention import kv_append
    g = torch.Generator(device="cuda").manual_seed(0)
    B, nq, nkv, D, S = 3, 8, 2, 128, 40
    qkv = torch.randn(B, nq + 2 * nkv, D, device="cuda", generator=g).to(torch.bfloat16)
    k, v = qkv[:, nq:nq + nkv], qkv[:, nq + nkv:]
    kc = torch.randn(B, nkv, S, D, device="cuda", generator=g).to(torch.bfloat16)
    vc = torch.randn(B, nkv, S, D, device="cuda", generator=g).to(torch.bfloat16)
    kr, vr = kc.clone(), vc.clone()
    cur = torch.tensor([17], device="cuda")
    kv_append(k, v, kc, vc, cur)
    kr.index_copy_(2, cur, k.reshape(B, nkv, 1, D))
    vr.index_copy_(2, cur, v.reshape(B, nkv, 1, D))
    torch.cuda.synchronize()
    assert torch.equal(kc, kr) and torch.equal(vc, vr)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["causal", "full", "window", "varlen", "gqa_tail"])
def test_flash_bwd_pipelined_matches_plain_gpu(case):
    """dK/dV and dQ kernels with LDS reads pipelined two MFMAs ahead (PIPE) give the plain kernels' gradients, and
    both match fp32 autograd."""
    from hcache_deepspeed_amd.ops import native
    from hcache_deepspeed_amd.ops.attention import flash_attn
    lib = native.kernels()
    torch.manual_seed(11)
    B, S, Hq, Hkv, D = 2, (701 if case == "gqa_tail" else 640), 8, 2, 128
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    kw = dict(causal=case != "full", window=100 if case == "window" else 0)
    grads = {}
    try:
        for pipe in (0, 1):
            lib.hds_attn_bwd_pipe(pipe)
            q.grad = k.grad = v.grad = None
            if case == "varlen":
                cu = torch.tensor([0, 333, 2 * S], device="cuda", dtype=torch.int32)
                o = flash_attn(q.reshape(-1, Hq, D), k.reshape(-1, Hkv, D), v.reshape(-1, Hkv, D), causal=True,
                               cu_seqlens=cu).view(B, S, Hq, D)
            else:
                o = flash_attn(q, k, v, **kw)
            o.backward(do)
            grads[pipe] = [t.grad.float().clone() for t in (q, k, v)]
    finally:
        lib.hds_attn_bwd_pipe(1)
    for a, b in zip(grads[0], grads[1]):
        assert (a - b).abs().max().item() <= 2e-2 * max(1.0, a.abs().max().item()), case
    if case in ("causal", "full", "gqa_tail"):
        qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
        kk, vv = kf.repeat_interleave(4, 2), vf.repeat_interleave(4, 2)
        s = torch.einsum("bqhd,bkhd->bhqk", qf, kk) / D**0.5
        if kw["causal"]:
            i = torch.arange(S, device="cuda")
            s = s.masked_fill(i[None, :] > i[:, None], float("-inf"))
        ref = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), vv)
        ref.backward(do.float())
        for g, r in zip(grads[1], (qf.grad, kf.grad, vf.grad)):
            rel = ((g - r).norm() / r.norm()).item()
            assert rel < 2e-2, (case, rel)


@pytest.mark.parametrize("lp_kind", ["bf16", "fp32", "fp32_alias", "fp16"])
def test_adam_flat_lp_out_dtypes_gpu(lp_kind):
    """The flat optimizer kernels write a bf16 parameter copy; any other compute copy (fp32 training, fp16) must come
    out equal to the updated fp32 parameters, never a bf16 bit pattern written into a wider buffer."""
    from hcache_deepspeed_amd.ops.optimizers import adam_flat
    torch.manual_seed(0)
    n = 10_000 + 3
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    ref_p = p.clone().cpu()
    if lp_kind == "fp32_alias":
        lp = p
    else:
        lp = torch.zeros(n, device="cuda", dtype={"bf16": torch.bfloat16, "fp32": torch.float32,
                                                  "fp16": torch.float16}[lp_kind])
    adam_flat(p, g, m, v, 1, 1e-2, lp_out=lp, weight_decay=0.01)
    gc = g.cpu()
    mm = 0.1 * gc
    vv = 0.001 * gc * gc
    upd = (mm / 0.1) / ((vv / 0.001).sqrt() + 1e-8) + 0.01 * ref_p
    want = ref_p - 1e-2 * upd
    torch.testing.assert_close(p.cpu(), want, rtol=1e-5, atol=1e-6)
    tol = {"bf16": 1e-2, "fp16": 1e-3}.get(lp_kind, 1e-6)
    torch.testing.assert_close(lp.float().cpu(), want, rtol=tol, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["causal", "full", "window", "varlen", "gqa_odd"])
def test_flash_bwd_dq_w64_matches_gpu(case):
    """Backward dQ variant 1 (one wave per SIMD, 64 query rows per wave, flash_attn_bwd_w64.hip) against variant 0 and
    the fp32 autograd reference; dK / dV come from the same kernel either way and must not move."""
    from hcache_deepspeed_amd.ops import native
    from hcache_deepspeed_amd.ops.attention import flash_attn
    lib = native.kernels()
    torch.manual_seed(11)
    B, S, Hq, Hkv, D = (2, 700, 8, 2, 128) if case != "gqa_odd" else (1, 333, 6, 3, 128)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    kw = dict(causal=case != "full", window=100 if case == "window" else 0)
    grads = {}
    try:
        for var in (0, 1):
            assert lib.hds_attn_bwd_dq_variant(var) == 0
            qg, kg, vg = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
            if case == "varlen":
                cu = torch.tensor([0, 333, 2 * S], device="cuda", dtype=torch.int32)
                o = flash_attn(qg.reshape(-1, Hq, D), kg.reshape(-1, Hkv, D), vg.reshape(-1, Hkv, D),
                               causal=True, cu_seqlens=cu).reshape(B, S, Hq, D)
            else:
                o = flash_attn(qg, kg, vg, **kw)
            o.backward(do)
            torch.cuda.synchronize()
            grads[var] = (qg.grad, kg.grad, vg.grad)
    finally:
        lib.hds_attn_bwd_dq_variant(int(os.environ.get("HDS_ATTN_DQ_VAR", "0")))
    dq0, dq1 = grads[0][0].float(), grads[1][0].float()
    assert torch.isfinite(dq1).all()
    rel = ((dq1 - dq0).norm() / dq0.norm()).item()
    assert rel < 1e-2, rel
    assert torch.equal(grads[0][1], grads[1][1]) and torch.equal(grads[0][2], grads[1][2])
    if case in ("causal", "full", "window"):
        G = Hq // Hkv
        qf, kf, vf = (t.float().transpose(1, 2).requires_grad_(True) for t in (q, k.repeat_interleave(G, 2),
                                                                                 v.repeat_interleave(G, 2)))
        s = qf @ kf.transpose(-1, -2) / D**0.5
        i = torch.arange(S, device="cuda")
        mask = torch.zeros(S, S, dtype=torch.bool, device="cuda")
        if kw["causal"]:
            mask |= i[None, :] > i[:, None]
        if kw["window"]:
            mask |= i[None, :] <= i[:, None] - kw["window"]
        ref = torch.softmax(s.masked_fill(mask, float("-inf")), -1) @ vf
        ref.backward(do.float().transpose(1, 2))
        dq_ref = qf.grad.transpose(1, 2)
        rel_ref = ((dq1 - dq_ref).norm() / dq_ref.norm()).item()
        assert rel_ref < 2e-2, rel_ref
