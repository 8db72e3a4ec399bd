"""Inference-v2 module registry + heuristics (reference inference/v2/modules, tests/unit/inference/v2/modules
strategy: each implementation against a torch reference; quantized linears within their format's error)."""
import pytest
import torch

from hcache_deepspeed_amd.inference.v2 import build_engine_from_model
from hcache_deepspeed_amd.inference.v2.modules import (DSLinearBase, DSLinearConfig, DSLinearRegistry, DSMoEConfig,
                                                       DSNormConfig, ConfigBundle, instantiate_linear,
                                                       instantiate_moe, instantiate_pre_norm)
from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny


def test_registry_selection_and_errors():
    assert type(instantiate_linear(DSLinearConfig(64, 32))).__name__ == "BlasFPLinear"
    q = instantiate_linear(DSLinearConfig(64, 32), type("EC", (), {"quantization": {"quantization_mode": "wf6af16"}}))
    assert q.name() == "quantized_wf6af16_linear"
    assert instantiate_linear(DSLinearConfig(64, 32, quantization_mode="int4")).name() == "quantized_int_linear"
    # shapes the packed kernels cannot take fall back to bf16
    assert instantiate_linear(DSLinearConfig(40, 32, quantization_mode="int8")).name() == "blas_fp_linear"
    with pytest.raises(ValueError):
        instantiate_linear(DSLinearConfig(64, 32, quantization_mode="nf4"))
    with pytest.raises(KeyError):
        DSLinearRegistry.instantiate_config(ConfigBundle("nope", DSLinearConfig(8, 8)))
    with pytest.raises(TypeError):
        DSLinearRegistry.register_module(int)
    assert "blas_fp_linear" in DSLinearRegistry.supporting(DSLinearConfig(64, 64))

    @DSLinearRegistry.register_module
    class _Custom(DSLinearBase):

        @staticmethod
        def name():
            return "custom_test_linear"

        def forward(self, x, w, b=None):
            return x @ w.t() * 2

    m = DSLinearRegistry.instantiate_config(ConfigBundle("custom_test_linear", DSLinearConfig(4, 4)))
    assert torch.equal(m(torch.ones(1, 4), torch.eye(4)), 2 * torch.ones(1, 4))
    del DSLinearRegistry.registry["custom_test_linear"]


@pytest.mark.parametrize("act", ["identity", "gelu", "relu", "silu_glu"])
@pytest.mark.parametrize("mode,tol", [(None, 1e-5), ("wf6af16", 0.08), ("int8", 0.02), ("int4", 0.2)])
def test_linear_implementations(act, mode, tol):
    torch.manual_seed(0)
    out = 96 if act.endswith("_glu") else 48
    x, w, b = torch.randn(5, 64), torch.randn(out, 64) * 0.2, torch.randn(out) * 0.1
    lin = instantiate_linear(DSLinearConfig(64, out, activation=act, quantization_mode=mode, group_size=32))
    y = lin(x, lin.transform_param(w), b)
    ref = x @ w.t() + b
    if act == "silu_glu":
        g, u = ref.chunk(2, -1)
        ref = torch.nn.functional.silu(g) * u
    elif act != "identity":
        ref = getattr(torch.nn.functional, act)(ref)
    err = (y.float() - ref).norm() / ref.norm()
    assert err < tol, (mode, act, float(err))


def test_pre_norm_and_moe_modules():
    torch.manual_seed(0)
    n = instantiate_pre_norm(DSNormConfig(32, "rms", 1e-6))
    r, h, g = torch.randn(4, 32), torch.randn(4, 32), torch.rand(32) + 0.5
    r2, y = n(r, h, g)
    s = r + h
    assert torch.allclose(r2, s) and torch.allclose(y, s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + 1e-6) * g,
                                                    atol=1e-5)
    moe = instantiate_moe(DSMoEConfig(32, 16, 4, 2, "silu_glu", True))
    x = torch.randn(6, 32)
    rw, w13, w2 = torch.randn(4, 32), torch.randn(4, 32, 32) * 0.2, torch.randn(4, 32, 16) * 0.2
    y = moe(x, rw, w13, w2)
    p = torch.softmax(x @ rw.t(), -1)
    tw, ti = p.topk(2, -1)
    tw = tw / tw.sum(-1, keepdim=True)
    ref = torch.zeros_like(x)
    for t in range(6):
        for j in range(2):
            e = int(ti[t, j])
            gu = w13[e] @ x[t]
            ref[t] += tw[t, j] * (w2[e] @ (torch.nn.functional.silu(gu[:16]) * gu[16:]))
    assert torch.allclose(y, ref, atol=1e-4), (y - ref).abs().max()


@pytest.mark.parametrize("mode,tol", [("wf6af16", 0.15), ("int8", 0.05)])
def test_quantized_engine_matches_bf16(mode, tol, tmp_path):
    from hcache_deepspeed_amd.inference.v2.engine import build_engine_from_ds_checkpoint
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(head_dim=64, hidden_size=128, intermediate_size=256, vocab_size=101,
                              num_attention_heads=2, num_key_value_heads=1, num_hidden_layers=2)).eval()
    base = dict(dtype="fp32", state_manager={"max_context": 256, "kv_block_size": 64})
    ids = torch.randint(0, 101, (20, ), generator=torch.Generator().manual_seed(2))
    ref, _ = build_engine_from_model(m, base, device=torch.device("cpu"), num_kv_blocks=8).put([1], [ids])
    eng = build_engine_from_model(m, {**base, "quantization": {"quantization_mode": mode}},
                                  device=torch.device("cpu"), num_kv_blocks=8)
    from hcache_deepspeed_amd.inference.v2.modules.implementations import _PackedWeight
    assert isinstance(eng._model.layers[0].w["qkv.w"], _PackedWeight)
    got, _ = eng.put([1], [ids])
    err = (got - ref).norm() / ref.norm()
    assert err < tol, float(err)
    # serialize / reload keeps the packed weights
    eng.serialize(str(tmp_path))
    eng2 = build_engine_from_ds_checkpoint(str(tmp_path), {**base, "quantization": {"quantization_mode": mode}},
                                           device=torch.device("cpu"), num_kv_blocks=8)
    got2, _ = eng2.put([1], [ids])
    assert torch.equal(got, got2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,tol", [(None, 0.03), ("wf6af16", 0.15), ("int8", 0.06)])
def test_quantized_engine_gpu(mode, tol):
    """bf16 engine on the MI355X: decode steps run the FP6 / INT8 HIP GEMVs, prefill the dequant + GEMM path."""
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(head_dim=128, hidden_size=256, intermediate_size=512, vocab_size=211,
                              num_attention_heads=2, num_key_value_heads=1, num_hidden_layers=2)).eval()
    dev = torch.device("cuda")
    ids = torch.randint(0, 211, (40, ), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        full = m(torch.cat([ids, ids[:3]])[None]).float()
    cfg = dict(dtype="bf16", state_manager={"max_context": 256, "kv_block_size": 64})
    if mode:
        cfg["quantization"] = {"quantization_mode": mode}
    eng = build_engine_from_model(m, cfg, device=dev, num_kv_blocks=8)
    lg, _ = eng.put([1], [ids])
    outs = [lg[0].float().cpu()]
    for j in range(3):
        lg, _ = eng.put([1], [ids[j:j + 1]], capture_latents=False)
        outs.append(lg[0].float().cpu())
    want = full[[39, 40, 41, 42]]
    err = (torch.stack(outs) - want).norm() / want.norm()
    assert err < tol, float(err)
