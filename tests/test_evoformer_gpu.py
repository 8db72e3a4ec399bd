"""Evoformer attention HIP forward (csrc/kernels/evoformer.hip) vs an fp32 torch softmax reference; the backward
(chunked recompute from the kernel's LSE) vs autograd of the reference (reference
tests/unit/ops/deepspeed4science/test_DS4Sci_EvoformerAttention.py)."""
import math

import pytest
import torch

from hcache_deepspeed_amd.ops.deepspeed4science import DS4Sci_EvoformerAttention


def _ref(q, k, v, b1, b2):
    qh, kh, vh = (x.float().transpose(-2, -3) for x in (q, k, v))
    s = torch.matmul(qh, kh.transpose(-1, -2)) / math.sqrt(q.shape[-1])
    if b1 is not None:
        s = s + b1.float()
    if b2 is not None:
        s = s + b2.float()
    return torch.matmul(torch.softmax(s, -1), vh).transpose(-2, -3)


@pytest.mark.gpu
@pytest.mark.parametrize("D", [32, 64, 128])
@pytest.mark.parametrize("L", [70, 256])
@pytest.mark.parametrize("bias_dtype", [torch.bfloat16, torch.float32])
def test_evoformer_fwd_bwd_hip(cuda, D, L, bias_dtype):
    torch.manual_seed(0)
    B, N, H = 1, 5, 4
    q, k, v = (torch.randn(B, N, L, H, D, device=cuda, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    b1 = torch.randn(B, N, 1, 1, L, device=cuda, dtype=bias_dtype) * 0.5
    b1[..., -7:] = -1e9
    b1.requires_grad_(True)
    b2 = torch.randn(B, 1, H, L, L, device=cuda, dtype=bias_dtype).requires_grad_(True)
    out = DS4Sci_EvoformerAttention(q, k, v, [b1, b2])
    ref = _ref(q, k, v, b1, b2)
    assert out.dtype == torch.bfloat16
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    g = torch.randn_like(out)
    assert out.grad_fn is not None
    ga = torch.autograd.grad(out, (q, k, v, b1, b2), g)
    gb = torch.autograd.grad(ref, (q, k, v, b1, b2), g.float())
    for x, y in zip(ga, gb):
        err = (x.float() - y).abs().max().item()
        assert err <= 5e-2 * max(1.0, y.abs().max().item()), err


@pytest.mark.gpu
def test_evoformer_no_bias_hip(cuda):
    torch.manual_seed(1)
    q, k, v = (torch.randn(2, 3, 96, 2, 32, device=cuda, dtype=torch.bfloat16) for _ in range(3))
    out = DS4Sci_EvoformerAttention(q, k, v, [])
    torch.testing.assert_close(out.float(), _ref(q, k, v, None, None), atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
def test_evoformer_backward_runs_hip_kernels(cuda, monkeypatch):
    """The GPU backward is the HIP one (no chunked torch recompute)."""
    from hcache_deepspeed_amd.ops.deepspeed4science import evoformer_attn as ev
    called = []
    orig = ev._hip_backward
    monkeypatch.setattr(ev, "_hip_backward", lambda *a, **k: called.append(1) or orig(*a, **k))
    q, k, v = (torch.randn(1, 2, 64, 2, 32, device=cuda, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    DS4Sci_EvoformerAttention(q, k, v, []).sum().backward()
    assert called and q.grad is not None and torch.isfinite(q.grad.float()).all()
