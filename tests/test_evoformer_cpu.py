"""Evoformer attention (pair bias + MSA mask) vs a direct fp32 softmax reference, outputs and all gradients.

Reference test analogue: tests/unit/ops/deepspeed4science/test_DS4Sci_EvoformerAttention.py (compares against an
eager ``attention_reference`` with both biases, forward and backward).
"""
import math

import pytest
import torch

import hcache_deepspeed_amd.ops.deepspeed4science.evoformer_attn as ev
from hcache_deepspeed_amd.ops.deepspeed4science import DS4Sci_EvoformerAttention


def _ref(q, k, v, b1, b2):
    qh, kh, vh = (x.transpose(-2, -3) for x in (q, k, v))
    s = torch.matmul(qh, kh.transpose(-1, -2)) / math.sqrt(q.shape[-1]) + b1 + b2
    return torch.matmul(torch.softmax(s, -1), vh).transpose(-2, -3)


@pytest.mark.parametrize("chunk_bytes", [256 << 20, 4096])
def test_evoformer_matches_reference(chunk_bytes, monkeypatch):
    monkeypatch.setattr(ev, "_CHUNK_BYTES", chunk_bytes)  # 4096 forces many query chunks
    torch.manual_seed(0)
    B, N, L, H, D = 1, 3, 40, 2, 16
    q, k, v = (torch.randn(B, N, L, H, D, requires_grad=True) for _ in range(3))
    b1 = torch.zeros(B, N, 1, 1, L)
    b1[..., -4:] = -1e9
    b1.requires_grad_(True)
    b2 = torch.randn(B, 1, H, L, L, requires_grad=True)
    out = DS4Sci_EvoformerAttention(q, k, v, [b1, b2])
    ref = _ref(q, k, v, b1, b2)
    assert torch.allclose(out, ref, atol=1e-5)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, (q, k, v, b1, b2), g)
    gb = torch.autograd.grad(ref, (q, k, v, b1, b2), g)
    for x, y in zip(ga, gb):
        assert torch.allclose(x, y, atol=1e-4), (x - y).abs().max()


def test_evoformer_bias_optional():
    torch.manual_seed(1)
    q, k, v = (torch.randn(2, 2, 20, 4, 8) for _ in range(3))
    out = DS4Sci_EvoformerAttention(q, k, v, [])
    assert torch.allclose(out, _ref(q, k, v, 0.0, 0.0), atol=1e-5)
    with pytest.raises(AssertionError):
        DS4Sci_EvoformerAttention(q, k, v, [torch.zeros(2, 2, 20)])
