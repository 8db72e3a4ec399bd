"""Stacked-expert GEMMs on MI355X at Mixtral-8x7B width: the per-expert 2-D GEMM path (parallel/moe.py
``expert_linear``) against an fp32 reference, forward and both gradients. The batched hipBLASLt form of the
down projection failed on this shape (HIPBLAS_STATUS_INTERNAL_ERROR, then an illegal access in the fallback)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("E,C,N,K", [(8, 1280, 4096, 14336), (8, 1280, 28672, 4096), (4, 96, 256, 512)])
def test_expert_linear_matches_fp32(E, C, N, K):
    from hcache_deepspeed_amd.parallel.moe import expert_linear
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.randn(E, C, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(E, N, K, device="cuda", generator=g) * K**-0.5).to(torch.bfloat16).requires_grad_(True)
    y = expert_linear(x, w)
    dy = torch.randn(E, C, N, device="cuda", generator=g).to(torch.bfloat16)
    y.backward(dy)
    torch.cuda.synchronize()
    for e in (0, E - 1):
        xf, wf, dyf = x[e].detach().float(), w[e].detach().float(), dy[e].float()
        ref = xf @ wf.t()
        rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()  # noqa: E731
        assert rel(y[e], ref) < 1e-2
        assert rel(x.grad[e], dyf @ wf) < 1e-2
        assert rel(w.grad[e], dyf.t() @ xf) < 1e-2


def test_mixtral_layer_full_width_step():
    """One full-width Mixtral decoder layer (8 experts x 14336, top-2) forward + backward at S=4096."""
    from hcache_deepspeed_amd.models.mixtral import MixtralForCausalLM, mixtral_8x7b
    torch.manual_seed(0)
    m = MixtralForCausalLM(mixtral_8x7b(num_hidden_layers=1)).cuda().to(torch.bfloat16)
    x = torch.randint(0, 32000, (1, 4096), device="cuda")
    loss = m(x, labels=x)
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()
    g = m.layers[0].block_sparse_moe.deepspeed_moe.experts.w2.grad
    assert g is not None and torch.isfinite(g.float()).all().item() and g.abs().sum().item() > 0


def test_mixtral_engine_direct_expert_wgrad_matches():
    """Stacked expert weight gradients written in place into the ZeRO gradient buffer (per-expert GEMMs with
    out=slice) train the same trajectory as the dense AccumulateGrad path (``mi355x.direct_wgrad: false``),
    with gradient accumulation over 2 micro-steps."""
    import os
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.mixtral import MixtralForCausalLM, tiny_moe
    os.environ.setdefault("MASTER_PORT", "29571")
    res = {}
    for direct in (True, False):
        torch.manual_seed(0)
        m = MixtralForCausalLM(tiny_moe(hidden_size=256, intermediate_size=512, num_hidden_layers=2))
        cfg = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 3},
               "data_types": {"grad_accum_dtype": "bf16"}, "mi355x": {"direct_wgrad": direct}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        if direct:
            assert id(m.layers[0].block_sparse_moe.deepspeed_moe.experts.w13) in eng.optimizer._wgrad_ok
        g = torch.Generator(device="cuda").manual_seed(1)
        losses = []
        for _ in range(6):
            x = torch.randint(0, 512, (2, 256), device="cuda", generator=g)
            loss = eng(x, labels=x)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
        res[direct] = losses
    assert res[True] == pytest.approx(res[False], rel=2e-2, abs=2e-2), res
