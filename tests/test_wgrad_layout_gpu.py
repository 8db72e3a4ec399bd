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


@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
@pytest.mark.parametrize("T,I", [(256, 1024), (72, 136), (8, 8)])
def test_glu_transposed_outputs(act, T, I):
    """glu(transposed=True): y and its transpose from one kernel, d(gate|up) and its transpose from one kernel."""
    from hcache_deepspeed_amd.ops.activations import glu
    torch.manual_seed(0)
    gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    y = glu(gu, act, transposed=True)
    y0 = glu(gu.detach(), act)
    assert (y.detach().float() - y0.float()).abs().max().item() <= 1e-2 * y0.float().abs().max().item()
    assert torch.equal(y._hds_t, y.detach().t().contiguous())
    seen = {}

    class Probe(torch.autograd.Function):  # stands in for the gate|up projection: sees the gradient glu returns

        @staticmethod
        def forward(ctx, t):
            return t.view_as(t)

        @staticmethod
        def backward(ctx, g):
            seen["g"], seen["gt"] = g, getattr(g, "_hds_t", None)
            return g

    src = gu.detach().clone().requires_grad_(True)
    d = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    glu(Probe.apply(src), act, transposed=True).backward(d)
    ref = gu.detach().clone().requires_grad_(True)
    glu(ref, act).backward(d)
    # same math as the plain kernel (a different kernel: fp contraction may differ by an ulp for gelu_tanh)
    assert (seen["g"].float() - ref.grad.float()).abs().max().item() <= 1e-2 * ref.grad.float().abs().max().item()
    assert seen["gt"] is not None and torch.equal(seen["gt"], seen["g"].t().contiguous())


@pytest.mark.parametrize("pre", ["xt", "dyt", "both"])
def test_wgrad_pretransposed_operands(pre, monkeypatch):
    from hcache_deepspeed_amd.ops import gemm
    monkeypatch.setattr(gemm, "_WGRAD_CHOICE", {})
    torch.manual_seed(0)
    dy = torch.randn(2048, 768, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(2048, 512, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = torch.empty(768, 512, device="cuda", dtype=torch.bfloat16)
    xt = x.t().contiguous() if pre in ("xt", "both") else None
    dyt = dy.t().contiguous() if pre in ("dyt", "both") else None
    gemm.wgrad(dy, None if xt is not None else x, out, accumulate=False, dyt=dyt, xt=xt)
    gemm.wgrad(dy, None if xt is not None else x, out, accumulate=True, dyt=dyt, xt=xt)
    assert (out.float() - 2 * ref).abs().max().item() <= 4e-2 * ref.abs().max().item()


def test_zero_linear_saves_transposed_input():
    """runtime/zero/linear: an input carrying _hds_t is saved as its transpose; gradients match F.linear's."""
    from hcache_deepspeed_amd.runtime.zero.linear import zero3_linear
    torch.manual_seed(0)
    x = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(384, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    xx = x * 1
    xx._hds_t = xx.detach().t().contiguous()
    y = zero3_linear(xx, w)
    dy = torch.randn_like(y)
    y.backward(dy)
    x2, w2 = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    torch.nn.functional.linear(x2, w2).backward(dy.float())
    for a, b in ((w.grad, w2.grad), (x.grad, x2.grad)):
        assert (a.float() - b).abs().max().item() <= 2e-2 * b.abs().max().item()
