"""DeepSpeedTransformerLayer (BERT encoder block) vs an eager fp32 torch block built from the same weights.

Reference test analogue: tests/unit/ops/accelerators/test_accelerator_forward.py / _backward.py (DS layer vs the
HF-style BertEncoder reference, pre- and post-LN, with attention masks, comparing outputs and gradients).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from hcache_deepspeed_amd.ops.transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer


def _ref(layer, x, mask):
    c = layer.config
    B, S, H = x.shape
    nh, d = c.heads, H // c.heads
    f = lambda t: t.float()  # noqa: E731
    ln = lambda t, w, b: F.layer_norm(t, (H, ), f(w), f(b), c.layer_norm_eps)  # noqa: E731

    def attn(h):
        qkv = F.linear(h, f(layer.attn_qkvw), f(layer.attn_qkvb)).view(B, S, 3, nh, d)
        q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
        s = q @ k.transpose(-1, -2) / math.sqrt(d)
        if mask is not None:
            s = s + mask
        return (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, H)

    xf = x.float()
    if c.pre_layer_norm:
        x1 = xf + F.linear(attn(ln(xf, layer.attn_nw, layer.attn_nb)), f(layer.attn_ow), f(layer.attn_ob))
        h = ln(x1, layer.norm_w, layer.norm_b)
        return x1 + F.linear(F.gelu(F.linear(h, f(layer.inter_w), f(layer.inter_b)), approximate="tanh"),
                             f(layer.output_w), f(layer.output_b))
    h = ln(xf + F.linear(attn(xf), f(layer.attn_ow), f(layer.attn_ob)), layer.attn_nw, layer.attn_nb)
    o = F.linear(F.gelu(F.linear(h, f(layer.inter_w), f(layer.inter_b)), approximate="tanh"), f(layer.output_w),
                 f(layer.output_b))
    return ln(h + o, layer.norm_w, layer.norm_b)


def _cfg(pre, H=64, heads=4):
    return DeepSpeedTransformerConfig(batch_size=2, hidden_size=H, heads=heads, attn_dropout_ratio=0.0,
                                      hidden_dropout_ratio=0.0, num_hidden_layers=2, initializer_range=0.02,
                                      pre_layer_norm=pre, layer_norm_eps=1e-12)


@pytest.mark.parametrize("pre", [True, False])
def test_transformer_layer_matches_reference(pre):
    torch.manual_seed(0)
    layer = DeepSpeedTransformerLayer(_cfg(pre))
    with torch.no_grad():
        for p in (layer.attn_nw, layer.norm_w):
            p.add_(torch.randn_like(p) * 0.1)
    x = torch.randn(2, 16, 64, requires_grad=True)
    mask = torch.zeros(2, 1, 1, 16)
    mask[1, ..., -3:] = -10000.0
    out = layer(x, mask)
    ref = _ref(layer, x, mask)
    assert torch.allclose(out, ref, atol=1e-4)
    g = torch.randn_like(out)
    params = [x] + list(layer.parameters())
    ga = torch.autograd.grad(out, params, g)
    gb = torch.autograd.grad(ref, params, g)
    for a, b in zip(ga, gb):
        assert torch.allclose(a, b, atol=1e-3), (a - b).abs().max()


@pytest.mark.gpu
def test_transformer_layer_gpu_flash_path():
    """bf16 on GPU, head_dim 128, no mask: HIP FlashAttention + fused LN / bias-GeLU kernels."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(1)
    layer = DeepSpeedTransformerLayer(_cfg(True, H=512, heads=4)).cuda().bfloat16()
    x = torch.randn(2, 256, 512, device="cuda").bfloat16().requires_grad_(True)
    out = layer(x)
    ref = _ref(layer, x, None)
    g = torch.randn_like(ref)
    ga = torch.autograd.grad(out, [x, layer.attn_qkvw, layer.inter_w], g.bfloat16())
    gb = torch.autograd.grad(ref, [x, layer.attn_qkvw, layer.inter_w], g)
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    assert rel(out, ref) < 2e-2
    for a, b in zip(ga, gb):
        assert rel(a, b) < 3e-2


@pytest.mark.gpu
@pytest.mark.parametrize("H,heads", [(768, 12), (512, 4)])
def test_transformer_layer_gpu_padding_mask(H, heads, monkeypatch):
    """BERT-base shape (head_dim 64) with a right-padding attention mask: the HIP FlashAttention runs with
    per-sequence lengths (the torch attention is disabled), valid rows match the fp32 masked reference."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hcache_deepspeed_amd.ops.transformer import transformer as TL
    calls = []
    real = TL.flash_attn

    def spy(*a, **k):
        calls.append(k.get("seq_lens"))
        return real(*a, **k)

    monkeypatch.setattr(TL, "flash_attn", spy)
    torch.manual_seed(2)
    layer = DeepSpeedTransformerLayer(_cfg(False, H=H, heads=heads)).cuda().bfloat16()
    B, S = 3, 128
    lens = [128, 50, 7]
    mask = torch.zeros(B, 1, 1, S, device="cuda")
    for b, L in enumerate(lens):
        mask[b, ..., L:] = -10000.0
    x = torch.randn(B, S, H, device="cuda").bfloat16().requires_grad_(True)
    out = layer(x, mask.bfloat16())
    assert calls and calls[0] is not None and calls[0].tolist() == lens  # HIP kernel with per-sequence lengths
    ref = _ref(layer, x, mask)
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    for b, L in enumerate(lens):
        assert rel(out[b, :L], ref[b, :L]) < 2e-2
