"""init_inference (v1 engine): kernel injection on HF models, weight-only quantization, AutoTP sharding on gloo,
HIP-graph replay on GPU (reference tests/unit/inference/test_inference.py strategy: compare the injected /
sharded model's logits against the unmodified HF model)."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed


def _hf_llama(seed=0):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(seed)
    cfg = LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)
    return LlamaForCausalLM(cfg).eval()


def _single_env():
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29623"))


def test_kernel_injection_matches_hf_cpu():
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.inference.injection import FusedGatedMLP, FusedRMSNorm
    _single_env()
    ref = _hf_llama()
    model = _hf_llama()
    x = torch.randint(0, 128, (2, 16))
    with torch.no_grad():
        want = ref(x).logits
    eng = ds.init_inference(model, dtype=torch.float32, replace_with_kernel_inject=True)
    assert eng.injected >= 2 * 2 + 1
    assert any(isinstance(m, FusedRMSNorm) for m in eng.module.modules())
    assert any(isinstance(m, FusedGatedMLP) for m in eng.module.modules())
    got = eng(x).logits
    assert torch.allclose(got, want, atol=2e-4, rtol=2e-4), (got - want).abs().max()
    # generate passes through to HF with injected blocks
    out = eng.generate(x[:1, :4], max_new_tokens=3, do_sample=False)
    ref_out = ref.generate(x[:1, :4], max_new_tokens=3, do_sample=False)
    assert torch.equal(out, ref_out)


def test_weight_only_quantization_cpu():
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.inference.injection import QuantizedLinear
    _single_env()
    ref = _hf_llama(1)
    model = _hf_llama(1)
    x = torch.randint(0, 128, (1, 8))
    with torch.no_grad():
        want = ref(x).logits
    # CPU: QuantizedLinear only wraps CUDA linears; build one directly
    lin = model.model.layers[0].mlp.down_proj
    ql = QuantizedLinear(lin, bits=8, group_size=64)
    h = torch.randn(3, lin.in_features)
    assert torch.allclose(ql(h), lin(h), atol=0.05, rtol=0.05)
    eng = ds.init_inference(model, dtype=torch.float32, quant={"enabled": True, "bits": 8})
    assert torch.allclose(eng(x).logits, want, atol=1e-4)  # CPU linears are left unquantized


def _tp(rank, world):
    import hcache_deepspeed_amd as ds
    ref = _hf_llama(2)
    model = _hf_llama(2)
    x = torch.randint(0, 128, (2, 12), generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        want = ref(x).logits
    eng = ds.init_inference(model, dtype=torch.float32, tensor_parallel={"tp_size": 2})
    q = eng.module.model.layers[0].self_attn.q_proj
    assert q.weight.shape[0] == 64 // 2
    got = eng(x).logits
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()


def test_autotp_inference_hf_llama_gloo():
    run_distributed(_tp, 2)


@pytest.mark.gpu
def test_kernel_injection_and_hip_graph_gpu():
    import hcache_deepspeed_amd as ds
    from transformers import LlamaConfig, LlamaForCausalLM
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _single_env()
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    ref = LlamaForCausalLM(cfg).eval().cuda().to(torch.bfloat16)
    model = LlamaForCausalLM(cfg).eval()
    model.load_state_dict(ref.state_dict())
    x = torch.randint(0, 512, (2, 256), device="cuda")
    with torch.no_grad():
        want = ref(x).logits.float()
    eng = ds.init_inference(model, dtype=torch.bfloat16, replace_with_kernel_inject=True, enable_cuda_graph=True)
    got = eng(x).logits.float()
    got2 = eng(x).logits.float()  # graph replay
    rel = (got - want).norm() / want.norm()
    assert rel < 2e-2, rel
    assert torch.equal(got, got2)
    eng_q = ds.init_inference(LlamaForCausalLM(cfg).eval(), dtype=torch.bfloat16, quant={"enabled": True, "bits": 8})
    assert any(type(m).__name__ == "QuantizedLinear" for m in eng_q.module.modules())


def _hybrid(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.runtime.hybrid_engine import DeepSpeedHybridEngine
    from tests.test_zero_cpu import TINY
    torch.manual_seed(0)
    ref = LlamaForCausalLM(tiny(**TINY))
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           "zero_optimization": {"stage": 3}, "hybrid_engine": {"enabled": True, "max_out_tokens": 8}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    assert isinstance(eng, DeepSpeedHybridEngine)
    prompt = torch.randint(0, 97, (1, 5), generator=torch.Generator().manual_seed(3))
    out = eng.generate(prompt, max_new_tokens=4)
    # reference greedy decode with the full (unsharded) model
    ids = prompt
    with torch.no_grad():
        for _ in range(4):
            nxt = ref(ids).view(1, ids.shape[1], -1)[:, -1].argmax(-1, keepdim=True)
            ids = torch.cat([ids, nxt], 1)
    assert torch.equal(out, ids)
    # parameters are partitioned again after generate, training continues
    u = eng.optimizer.units[0]
    assert u.full is None or u.persistent
    x = torch.randint(0, 97, (2, 12))
    loss = eng(x, labels=x)
    eng.backward(loss)
    eng.step()
    assert eng.latency_stats()["generate_calls"] == 1


def test_hybrid_engine_zero3_generate_gloo():
    run_distributed(_hybrid, 2)
