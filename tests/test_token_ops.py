"""Random-LTD token ops and NHWC bias-add fusions (csrc/kernels/token_ops.hip) against plain torch references.

Reference test model: tests/unit/ops/random_ltd (none upstream beyond the data-efficiency tests) and
tests/unit/ops/spatial/test_nhwc_bias_add.py (fused result == torch expression).
"""
import pytest
import torch

from hcache_deepspeed_amd.ops.random_ltd import (GatherTokens, ScatterTokens, gather_rows, scatter_rows,
                                                 slice_attention_mask, token_sort_)
from hcache_deepspeed_amd.ops.spatial import nhwc_bias_add


def _idx(B, S, R, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.stack([torch.randperm(S, generator=g)[:R].sort().values for _ in range(B)]).to(torch.int32).to(device)


def _autograd_check(device, dtype):
    B, S, R, H = 3, 40, 17, 64
    x = torch.randn(B, S, H, device=device, dtype=dtype, requires_grad=True)
    idx = _idx(B, S, R, device)
    _, part = GatherTokens.apply(x, idx, True)
    y = ScatterTokens.apply(x, part * 3.0, idx, True)
    w = torch.randn_like(y)
    (y * w).sum().backward()
    # reference: y = x with rows idx scaled by 3 -> dy/dx = w everywhere, 3w at idx rows
    xr = x.detach().float().clone().requires_grad_(True)
    m = torch.ones(B, S, 1, device=device)
    m[torch.arange(B, device=device)[:, None], idx.long()] = 3.0
    (xr * m * w.float()).sum().backward()
    assert torch.allclose(y.float(), (x.detach().float() * m), atol=1e-2, rtol=1e-2)
    assert torch.allclose(x.grad.float(), xr.grad, atol=2e-2, rtol=2e-2)


def test_gather_scatter_autograd_cpu():
    _autograd_check("cpu", torch.float32)


def test_token_sort_and_mask_cpu():
    k = torch.randint(0, 1000, (4, 37), dtype=torch.int32)
    ref = k.sort(-1).values
    assert torch.equal(token_sort_(k), ref)
    mask = torch.randn(2, 1, 12, 12)
    idx = _idx(2, 12, 5, "cpu")
    out = slice_attention_mask(mask, idx)
    for b in range(2):
        il = idx[b].long()
        assert torch.equal(out[b, 0], mask[b, 0][il][:, il])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gather_scatter_hip(dtype):
    B, S, R, H = 4, 512, 200, 4096
    x = torch.randn(B, S, H, device="cuda", dtype=dtype)
    idx = _idx(B, S, R, "cuda")
    g = gather_rows(x, idx)
    from hcache_deepspeed_amd.ops.random_ltd import _gather_ref, _scatter_ref
    assert torch.equal(g, _gather_ref(x, idx))
    part = torch.randn(B, R, H, device="cuda", dtype=dtype)
    assert torch.equal(scatter_rows(x, part, idx), _scatter_ref(x, part, idx))
    _autograd_check("cuda", dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 1000, 4096, 16384])
def test_token_sort_hip(n):
    k = torch.randint(-5000, 5000, (6, n), dtype=torch.int32, device="cuda")
    ref = k.sort(-1).values
    assert torch.equal(token_sort_(k.clone()), ref)


@pytest.mark.gpu
def test_slice_mask_hip():
    L, B, S, R = 2, 3, 256, 100
    idx = torch.stack([_idx(B, S, R, "cuda", seed=s) for s in range(L)])
    for Bm in (1, B):
        mask = torch.randn(Bm, 1, S, S, device="cuda", dtype=torch.bfloat16)
        out = slice_attention_mask(mask, idx)
        ref = slice_attention_mask(mask.cpu(), idx.cpu())
        assert out.shape == (L, B, 1, R, R)
        assert torch.equal(out.cpu(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_nhwc_bias_add_hip(mode, dtype):
    a = torch.randn(2, 16, 16, 320, device="cuda", dtype=dtype)
    b = torch.randn(320, device="cuda", dtype=dtype)
    o = torch.randn_like(a) if mode >= 1 else None
    ob = torch.randn(320, device="cuda", dtype=dtype) if mode == 2 else None
    ref = a.float() + b.float()
    if o is not None:
        ref = ref + o.float()
    if ob is not None:
        ref = ref + ob.float()
    out = nhwc_bias_add(a, b, o, ob)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert torch.allclose(out.float(), ref, atol=tol, rtol=tol)
