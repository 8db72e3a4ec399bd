"""Serving-engine parity against HuggingFace ``transformers`` for every supported model family.

Reference parity: inference/v2/engine_factory.py:69-130 (llama, mistral, mixtral, qwen, qwen2, qwen2_moe,
phi, phi3, falcon, opt policies) and tests/unit/inference/v2/ (which only exercises kernels/modules; the
reference pins no end-to-end logits). Here tiny random-init HF models are the oracle: ragged prefill of
two sequences, decode, and HCache restore_kv from latents must all reproduce ``model(ids).logits``.
Qwen (v1) needs remote code that is not importable here: its converter is "parity unpinned".
"""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from hcache_deepspeed_amd.inference.v2 import build_engine_from_hf_model  # noqa: E402

V = 151


def _families(H=64):
    t = transformers

    def _base(**kw):
        d = dict(vocab_size=V, hidden_size=H, intermediate_size=2 * H, num_hidden_layers=2, num_attention_heads=4,
                 num_key_value_heads=2, max_position_embeddings=256)
        d.update(kw)
        return d

    return {
        "llama": lambda: t.LlamaForCausalLM(t.LlamaConfig(**_base())),
        "mistral": lambda: t.MistralForCausalLM(t.MistralConfig(**_base(sliding_window=None))),
        "mixtral": lambda: t.MixtralForCausalLM(t.MixtralConfig(**_base(num_local_experts=4,
                                                                          num_experts_per_tok=2))),
        "qwen2": lambda: t.Qwen2ForCausalLM(t.Qwen2Config(**_base())),
        "qwen2_moe": lambda: t.Qwen2MoeForCausalLM(t.Qwen2MoeConfig(**_base(
            num_experts=4, num_experts_per_tok=2, moe_intermediate_size=H // 4 * 3, shared_expert_intermediate_size=H * 3 // 2,
            decoder_sparse_step=1, mlp_only_layers=[]))),
        "phi3": lambda: t.Phi3ForCausalLM(t.Phi3Config(**_base(pad_token_id=0))),
        "phi": lambda: t.PhiForCausalLM(t.PhiConfig(**_base(num_key_value_heads=4, partial_rotary_factor=0.5))),
        "falcon": lambda: t.FalconForCausalLM(t.FalconConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2,
                                                             num_attention_heads=4, multi_query=True,
                                                             parallel_attn=True, bias=False, alibi=False,
                                                             new_decoder_architecture=False)),
        "falcon_new": lambda: t.FalconForCausalLM(t.FalconConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2,
                                                                 num_attention_heads=4, num_kv_heads=2,
                                                                 new_decoder_architecture=True, bias=False,
                                                                 alibi=False)),
        "opt": lambda: t.OPTForCausalLM(t.OPTConfig(vocab_size=V, hidden_size=H, num_hidden_layers=2,
                                                    num_attention_heads=4, ffn_dim=2 * H, max_position_embeddings=256,
                                                    word_embed_proj_dim=H)),
    }


def _randomize(m):
    # HF zero-inits biases and some norms; perturb everything so the converter is actually exercised.
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() == 1:
                base = 1.0 if ("norm" in n or "ln" in n) and n.endswith("weight") else 0.0
                p.copy_(base + 0.1 * torch.randn(p.shape, generator=g))
    return m


@pytest.mark.parametrize("family", sorted(_families().keys()))
@pytest.mark.parametrize("latent_mode", ["hidden", "kv"])
def test_family_parity(family, latent_mode):
    torch.manual_seed(0)
    m = _randomize(_families()[family]().float().eval())
    eng = build_engine_from_hf_model(m, {"dtype": "fp32", "latent_mode": latent_mode,
                                         "state_manager": {"max_context": 256, "kv_block_size": 16}},
                                     device=torch.device("cpu"), num_kv_blocks=64)
    g = torch.Generator().manual_seed(1)
    p1 = torch.randint(0, V, (37, ), generator=g)
    p2 = torch.randint(0, V, (20, ), generator=g)
    cont = torch.randint(0, V, (4, ), generator=g)
    with torch.no_grad():
        ref1 = m(torch.cat([p1, cont])[None]).logits[0].float()
        ref2 = m(p2[None]).logits[0].float()
    tol = 2e-4
    logits, lats = eng.put([1, 2], [p1, p2])
    assert torch.allclose(logits[0], ref1[36], atol=tol, rtol=tol), (logits[0] - ref1[36]).abs().max()
    assert torch.allclose(logits[1], ref2[-1], atol=tol, rtol=tol), (logits[1] - ref2[-1]).abs().max()
    # decode one token on the live cache, then evict + restore from latents and continue
    lg, _ = eng.put([1], [cont[:1]], capture_latents=False)
    assert torch.allclose(lg[0], ref1[37], atol=tol, rtol=tol)
    eng.flush(1)
    logits, lats = eng.put([1], [p1])
    eng.evict(1)
    eng.restore_kv([1], [p1], [lats[0]])
    for j in range(cont.numel()):
        lg, _ = eng.put([1], [cont[j:j + 1]], capture_latents=False)
        assert torch.allclose(lg[0], ref1[37 + j], atol=tol, rtol=tol), (family, j)


@pytest.mark.parametrize("family", ["llama", "mixtral", "falcon"])
def test_hf_checkpoint_dir_and_serialize_roundtrip(family, tmp_path):
    from hcache_deepspeed_amd.inference.v2 import build_engine_from_ds_checkpoint, build_hf_engine
    torch.manual_seed(0)
    m = _randomize(_families()[family]().float().eval())
    m.save_pretrained(str(tmp_path / "hf"))
    cfg = {"dtype": "fp32", "state_manager": {"max_context": 256, "kv_block_size": 16}}
    eng = build_hf_engine(str(tmp_path / "hf"), cfg, device=torch.device("cpu"))
    ids = torch.randint(0, V, (19, ), generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        ref = m(ids[None]).logits[0, -1].float()
    lg, _ = eng.put([1], [ids])
    assert torch.allclose(lg[0], ref, atol=2e-4, rtol=2e-4)
    eng.serialize(str(tmp_path / "ds"))
    eng2 = build_engine_from_ds_checkpoint(str(tmp_path / "ds"), cfg, device=torch.device("cpu"), num_kv_blocks=32)
    lg2, _ = eng2.put([1], [ids])
    assert torch.allclose(lg2[0], lg[0], atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("family,H", [("llama", 512), ("mixtral", 512), ("qwen2_moe", 512), ("phi3", 512),
                                      ("phi", 512), ("falcon_new", 512), ("opt", 512),
                                      # the families' real head dims: Phi 80 (partial rotary 32), Phi-3 96,
                                      # Falcon / OPT 64, and a 256-wide head
                                      ("phi", 320), ("phi3", 384), ("falcon", 256), ("opt", 256), ("llama", 1024)])
def test_family_parity_gpu(family, H, monkeypatch):
    """HIP paged attention / fused RoPE+KV-scatter path (head_dim H/4) on every block structure; the torch
    reference serving path is disabled so a silent fallback fails the test."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hcache_deepspeed_amd.ops import paged as P
    real = P.paged_attention

    def hip_only(q, *a, **k):
        assert q.is_cuda
        return real(q, *a, **k)

    monkeypatch.setattr(P, "paged_attention", hip_only)
    m = _families(H=H)[family]()
    torch.manual_seed(0)
    m = _randomize(m.float().eval())
    eng = build_engine_from_hf_model(m, {"dtype": "bf16", "latent_mode": "kv",
                                         "state_manager": {"max_context": 256, "kv_block_size": 64}},
                                     device=torch.device("cuda"), num_kv_blocks=32)
    g = torch.Generator().manual_seed(1)
    p1 = torch.randint(0, V, (70, ), generator=g)
    cont = torch.randint(0, V, (3, ), generator=g)
    with torch.no_grad():
        ref = m(torch.cat([p1, cont])[None]).logits[0].float()
    logits, lats = eng.put([1], [p1])
    tol = 6e-2
    assert torch.allclose(logits[0].float().cpu(), ref[69], atol=tol, rtol=tol)
    eng.evict(1)
    eng.restore_kv([1], [p1], [lats[0]])
    for j in range(cont.numel()):
        lg, _ = eng.put([1], [cont[j:j + 1]], capture_latents=False)
        assert torch.allclose(lg[0].float().cpu(), ref[70 + j], atol=tol, rtol=tol), (family, j)
