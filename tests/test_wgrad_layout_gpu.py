"""Weight-gradient layout selection (ops/gemm.wgrad) and the HIP bf16 transpose against torch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("R,C,ld", [(64, 64, 64), (1000, 136, 136), (4096, 520, 1024), (8, 7, 8), (64, 128, 128),
                                    (200, 260, 264), (72, 129, 136), (4096, 4096, 4096)])
def test_transpose_matches_torch(R, C, ld, variant):
    from hcache_deepspeed_amd.ops.gemm import transpose2d
    base = torch.randn(R, ld, device="cuda", dtype=torch.bfloat16)
    x = base[:, :C]
    assert torch.equal(transpose2d(x, variant=variant), x.t().contiguous())


@pytest.mark.parametrize("layout", ["direct", "nt", "direct_sk2", "nt_sk2", "direct_b2", "nt_b2", "auto"])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_wgrad_layouts_match(layout, out_dtype, monkeypatch):
    from hcache_deepspeed_amd.ops import gemm
    monkeypatch.setattr(gemm, "_WGRAD_LAYOUT", layout)
    torch.manual_seed(0)
    dy = torch.randn(2048, 768, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(2048, 512, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = torch.empty(768, 512, device="cuda", dtype=out_dtype)
    gemm.wgrad(dy, x, out, accumulate=False)
    gemm.wgrad(dy, x, out, accumulate=True)
    err = (out.float() - 2 * ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() * 2, err


@pytest.mark.parametrize("layout", ["direct", "nt", "auto"])
def test_dgrad_layouts_match(layout, monkeypatch):
    from hcache_deepspeed_amd.ops import gemm
    monkeypatch.setattr(gemm, "_DGRAD_LAYOUT", layout)
    torch.manual_seed(0)
    dy = torch.randn(1024, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(768, 512, device="cuda", dtype=torch.bfloat16)
    ref = dy.float() @ w.float()
    got = gemm.dgrad(dy, w)
    assert (got.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    cache = {}
    for _ in range(2):  # the second call reuses the cached transposed weight
        assert torch.equal(gemm.dgrad(dy, w, cache=cache), got)
    out = torch.empty(1024, 512, device="cuda", dtype=torch.bfloat16)
    gemm.dgrad(dy, w, out=out)
    assert torch.equal(out, got)
