"""Grouped (MoE) GEMM (csrc/kernels/grouped_gemm.hip) and the dropless MoE FFN against fp32 torch references.

Reference test model: tests/unit/inference/v2/kernels/cutlass_ops/test_moe_gemm.py (grouped GEMM with ragged
per-expert token counts, including empty experts, vs per-expert torch matmuls).
"""
import pytest
import torch

from hcache_deepspeed_amd.ops.activations import glu
from hcache_deepspeed_amd.ops.grouped_gemm import expert_offsets, grouped_gemm, moe_ffn_dropless
from hcache_deepspeed_amd.ops.moe import moe_combine, moe_dispatch, topk_assign, topk_route


def _ref(x, w, counts):
    out, o = [], 0
    for e, c in enumerate(counts):
        out.append(x[o:o + c].float() @ w[e].float().t())
        o += c
    return torch.cat(out)


def _bmm_moe(x, logits, k, w13, w2):
    E, H = w13.shape[0], x.shape[1]
    ex, pos, w, C, _, _ = topk_route(logits, k, 1.0, 1, drop_tokens=False, use_rts=False, training=False)
    d = moe_dispatch(x, ex, pos, E, C).view(E, C, H)
    h = torch.bmm(d, w13.transpose(1, 2))
    y = torch.bmm(glu(h.reshape(E * C, -1), "silu").view(E, C, -1), w2.transpose(1, 2))
    return moe_combine(y.reshape(E * C, H), ex, pos, w, C)


def test_dropless_moe_matches_capacity_formulation_cpu():
    torch.manual_seed(0)
    T, H, I, E, k = 37, 16, 24, 4, 2
    x, logits = torch.randn(T, H), torch.randn(T, E)
    w13, w2 = torch.randn(E, 2 * I, H) * 0.1, torch.randn(E, H, I) * 0.1
    ex, pos, w, counts = topk_assign(logits, k)
    out = moe_ffn_dropless(x, ex, pos, w, counts, w13, w2, lambda h: glu(h, "silu"))
    torch.testing.assert_close(out, _bmm_moe(x, logits, k, w13, w2), atol=1e-5, rtol=1e-5)


def test_grouped_gemm_autograd_cpu():
    torch.manual_seed(1)
    counts = [5, 0, 9, 3]
    x = torch.randn(sum(counts), 8, requires_grad=True)
    w = torch.randn(4, 6, 8, requires_grad=True)
    y = grouped_gemm(x, w, expert_offsets(torch.tensor(counts)))
    g = torch.randn_like(y)
    (y * g).sum().backward()
    xr, wr = x.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    (_ref(xr, wr, counts) * g).sum().backward()
    torch.testing.assert_close(x.grad, xr.grad)
    torch.testing.assert_close(w.grad, wr.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("counts,N,K", [([300, 0, 1, 129, 128, 77], 256, 384), ([4096, 2048], 512, 1024),
                                        ([0, 0, 3], 256, 128), ([513, 255, 256, 1000], 768, 256)])
def test_grouped_gemm_hip(cuda, counts, N, K, variant):
    torch.manual_seed(2)
    E, T = len(counts), sum(counts)
    x = torch.randn(T, K, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(E, N, K, device=cuda, dtype=torch.bfloat16) / K**0.5
    y = grouped_gemm(x, w, expert_offsets(torch.tensor(counts, device=cuda)), variant=variant)
    ref = _ref(x, w, counts)
    assert y.dtype == torch.bfloat16
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
def test_grouped_gemm_backward_hip(cuda):
    torch.manual_seed(3)
    counts = [200, 57, 0, 311]
    x = torch.randn(sum(counts), 256, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(4, 384, 256, device=cuda, dtype=torch.bfloat16) / 16).requires_grad_(True)
    y = grouped_gemm(x, w, expert_offsets(torch.tensor(counts, device=cuda)))
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    xr, wr = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    (_ref(xr, wr, counts) * g.float()).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=3e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=5e-2, rtol=3e-2)


@pytest.mark.gpu
def test_dropless_moe_hip(cuda):
    torch.manual_seed(4)
    T, H, I, E, k = 333, 256, 384, 8, 2
    x = torch.randn(T, H, device=cuda, dtype=torch.bfloat16)
    logits = torch.randn(T, E, device=cuda)
    w13 = torch.randn(E, 2 * I, H, device=cuda, dtype=torch.bfloat16) / 16
    w2 = torch.randn(E, H, I, device=cuda, dtype=torch.bfloat16) / 20
    ex, pos, w, counts = topk_assign(logits, k)
    out = moe_ffn_dropless(x, ex, pos, w, counts, w13, w2, lambda h: glu(h, "silu"))
    ref = _bmm_moe(x.float().cpu(), logits.cpu(), k, w13.float().cpu(), w2.float().cpu())
    torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=3e-2)
