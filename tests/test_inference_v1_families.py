"""init_inference kernel injection across the reference's v1 container families (GPT-2, GPT-J, GPT-Neo,
GPT-NeoX, OPT, BLOOM, BERT; reference module_inject/containers/*.py and tests/unit/inference/test_inference.py):
the injected model's logits must match the unmodified HF model. CPU runs the fp32 torch fallbacks of the
same ops; the GPU test runs the HIP LayerNorm / bias+activation kernels in bf16. Random-init tiny configs
(no checkpoints are available offline)."""
import os

import pytest
import torch



def _single_env():
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29624"))


def _build(family, seed=0):
    import transformers as T
    torch.manual_seed(seed)
    common = dict(vocab_size=128)
    if family == "gpt2":
        m = T.GPT2LMHeadModel(T.GPT2Config(n_embd=64, n_layer=2, n_head=4, n_positions=64, **common))
    elif family == "gptj":
        m = T.GPTJForCausalLM(T.GPTJConfig(n_embd=64, n_layer=2, n_head=4, rotary_dim=8, n_positions=64, **common))
    elif family == "gpt_neo":
        m = T.GPTNeoForCausalLM(T.GPTNeoConfig(hidden_size=64, num_layers=2, num_heads=4,
                                               attention_types=[[["global", "local"], 1]], max_position_embeddings=64,
                                               window_size=16, **common))
    elif family == "gpt_neox":
        m = T.GPTNeoXForCausalLM(T.GPTNeoXConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                                 intermediate_size=256, max_position_embeddings=64, **common))
    elif family == "opt":
        m = T.OPTForCausalLM(T.OPTConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, ffn_dim=256,
                                         word_embed_proj_dim=64, max_position_embeddings=64, **common))
    elif family == "bloom":
        m = T.BloomForCausalLM(T.BloomConfig(hidden_size=64, n_layer=2, n_head=4, **common))
    elif family == "bert":
        m = T.BertForMaskedLM(T.BertConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                           intermediate_size=256, max_position_embeddings=64, **common))
    else:
        raise ValueError(family)
    return m.eval()


FAMILIES = ["gpt2", "gptj", "gpt_neo", "gpt_neox", "opt", "bloom", "bert"]


def _check(family, device, dtype, atol):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.inference.injection import FusedLayerNorm, LinearBiasAct
    _single_env()
    ref = _build(family).to(device=device, dtype=dtype)
    model = _build(family)
    x = torch.randint(0, 128, (2, 16), device=device)
    with torch.no_grad():
        want = ref(x).logits.float()
    eng = ds.init_inference(model, dtype=dtype, replace_with_kernel_inject=True)
    mods = list(eng.module.modules())
    assert sum(isinstance(m, FusedLayerNorm) for m in mods) >= 2 + 1, family
    assert sum(isinstance(m, LinearBiasAct) for m in mods) == 2, family
    got = eng(x).logits.float()
    err = (got - want).abs().max().item()
    assert err <= atol * max(1.0, want.abs().max().item()), (family, err)
    return eng


@pytest.mark.parametrize("family", FAMILIES)
def test_family_injection_matches_hf_cpu(family):
    eng = _check(family, "cpu", torch.float32, 2e-4)
    if family != "bert":  # generate passes through to HF with the injected blocks
        ref = _build(family)
        x = torch.randint(0, 128, (1, 5))
        out = eng.generate(x, max_new_tokens=3, do_sample=False)
        assert torch.equal(out, ref.generate(x, max_new_tokens=3, do_sample=False))


def test_activation_mapping():
    import torch.nn as nn
    from transformers.activations import ACT2FN
    from hcache_deepspeed_amd.inference.injection import _act_of
    assert _act_of(ACT2FN["gelu_new"]) == "gelu_tanh"
    assert _act_of(ACT2FN["gelu_pytorch_tanh"]) == "gelu_tanh"
    assert _act_of(ACT2FN["gelu"]) == "gelu"
    assert _act_of(ACT2FN["relu"]) == "relu"
    assert _act_of(ACT2FN["silu"]) == "silu"
    assert _act_of(nn.GELU(approximate="tanh")) == "gelu_tanh"
    assert _act_of(nn.Tanh()) is None


@pytest.mark.gpu
@pytest.mark.parametrize("family", FAMILIES)
def test_family_injection_matches_hf_gpu(family):
    from hcache_deepspeed_amd.ops import native
    native.kernels()  # the HIP path must be the one that runs
    _check(family, "cuda", torch.bfloat16, 6e-2)


GEN_FAMILIES = ["gptj", "gpt_neo", "bloom", "gpt_neox", "opt"]


def _gen_check(family, device, dtype):
    """Greedy generation through the KV cache (prefill + decode steps, left-padded batch) must reproduce HF."""
    import hcache_deepspeed_amd as ds
    _single_env()
    ref = _build(family).to(device=device, dtype=dtype)
    model = _build(family)
    x = torch.randint(3, 128, (2, 12), device=device)
    am = torch.ones_like(x)
    am[1, :4] = 0  # left padding of the second prompt
    x[1, :4] = 0
    kw = dict(max_new_tokens=6, do_sample=False, attention_mask=am, pad_token_id=0)
    with torch.no_grad():
        want = ref.generate(x, **kw)
    eng = ds.init_inference(model, dtype=dtype, replace_with_kernel_inject=True)
    if family in ("gptj", "gpt_neo", "bloom"):
        assert any(getattr(m, "_hds_container", False) for m in eng.module.modules()), family
    with torch.no_grad():
        got = eng.module.generate(x, **kw)
    return got, want


@pytest.mark.parametrize("family", GEN_FAMILIES)
def test_family_generate_matches_hf_cpu(family):
    got, want = _gen_check(family, "cpu", torch.float32)
    assert torch.equal(got, want), (family, got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("family", GEN_FAMILIES)
def test_family_generate_matches_hf_gpu(family):
    got, want = _gen_check(family, "cuda", torch.bfloat16)
    # bf16: greedy paths may split on near-ties after the first tokens; the first new tokens must agree
    assert torch.equal(got[:, :14], want[:, :14]), (family, got, want)
