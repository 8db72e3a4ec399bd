"""KV-cached generation (models/generation.py) against full-recompute greedy decoding, left-padded prompts,
tensor-parallel generation over gloo, and the hybrid engine's TP generate (reference hybrid_engine.py :168-272,
tests/unit/hybrid_engine strategy: generated tokens of the hybrid path equal the plain model's)."""
import torch

from tests.dist_utils import run_distributed

CFG = dict(vocab_size=97, hidden_size=64, intermediate_size=96, num_hidden_layers=2, num_attention_heads=4,
           num_key_value_heads=2, max_position_embeddings=64)


def _model(seed=0, **kw):
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(seed)
    return LlamaForCausalLM(tiny(**{**CFG, **kw})).eval()


def _greedy_ref(model, ids, n):
    with torch.no_grad():
        for _ in range(n):
            nxt = model(ids).view(ids.shape[0], ids.shape[1], -1)[:, -1].argmax(-1, keepdim=True)
            ids = torch.cat([ids, nxt], 1)
    return ids


def test_kv_generation_matches_recompute():
    from hcache_deepspeed_amd.models.generation import generate, supports_kv_generation
    m = _model()
    assert supports_kv_generation(m)
    prompt = torch.randint(0, 97, (3, 7), generator=torch.Generator().manual_seed(1))
    assert torch.equal(generate(m, prompt, max_new_tokens=9), _greedy_ref(m, prompt, 9))


def test_kv_generation_sliding_window():
    from hcache_deepspeed_amd.models.generation import generate
    m = _model(sliding_window=4)
    prompt = torch.randint(0, 97, (2, 6), generator=torch.Generator().manual_seed(2))
    assert torch.equal(generate(m, prompt, max_new_tokens=7), _greedy_ref(m, prompt, 7))


def test_kv_generation_left_padding():
    from hcache_deepspeed_amd.models.generation import generate
    m = _model()
    g = torch.Generator().manual_seed(4)
    a = torch.randint(1, 97, (1, 8), generator=g)
    b = torch.randint(1, 97, (1, 5), generator=g)
    batch = torch.cat([a, torch.cat([torch.zeros(1, 3, dtype=torch.long), b], 1)], 0)
    mask = torch.ones_like(batch)
    mask[1, :3] = 0
    out = generate(m, batch, attention_mask=mask, max_new_tokens=6)
    assert torch.equal(out[0], generate(m, a, max_new_tokens=6)[0])
    assert torch.equal(out[1, 3:], generate(m, b, max_new_tokens=6)[0])


def test_kv_generation_sampling_and_eos():
    from hcache_deepspeed_amd.models.generation import _sample, generate
    m = _model()
    prompt = torch.randint(0, 97, (4, 5), generator=torch.Generator().manual_seed(5))
    o1 = generate(m, prompt, max_new_tokens=6, do_sample=True, top_k=5, top_p=0.9, temperature=0.7,
                  generator=torch.Generator().manual_seed(0))
    o2 = generate(m, prompt, max_new_tokens=6, do_sample=True, top_k=5, top_p=0.9, temperature=0.7,
                  generator=torch.Generator().manual_seed(0))
    assert torch.equal(o1, o2) and o1.shape == (4, 11)
    # top-k=1 sampling is greedy
    assert torch.equal(generate(m, prompt, max_new_tokens=4, do_sample=True, top_k=1), _greedy_ref(m, prompt, 4))
    # nucleus keeps the smallest prefix reaching top_p
    logits = torch.log(torch.tensor([[0.5, 0.3, 0.15, 0.05]]))
    draws = {int(_sample(logits, True, 1.0, 0, 0.7, torch.Generator().manual_seed(s))) for s in range(50)}
    assert draws == {0, 1}
    # eos: rows stop and are padded
    greedy = _greedy_ref(m, prompt, 6)
    eos = int(greedy[0, 6])
    out = generate(m, prompt, max_new_tokens=6, eos_token_id=eos, pad_token_id=0)
    assert int(out[0, 6]) == eos and bool((out[0, 7:] == 0).all())


def _tp_generate(rank, world):
    from hcache_deepspeed_amd import comm as dist
    from hcache_deepspeed_amd.models.generation import generate
    m = _model()
    prompt = torch.randint(0, 97, (2, 6), generator=torch.Generator().manual_seed(7))
    want = generate(m, prompt, max_new_tokens=8)
    got = generate(m, prompt, tp_group=dist.new_group(list(range(world))), max_new_tokens=8)
    assert torch.equal(got, want), (got, want)


def test_tp_generation_gloo():
    run_distributed(_tp_generate, 2)


def _hybrid_tp(rank, world):
    import hcache_deepspeed_amd as ds
    m = _model()
    ref = _model()
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           "zero_optimization": {"stage": 3},
           "hybrid_engine": {"enabled": True, "max_out_tokens": 8, "inference_tp_size": 2}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    prompt = torch.randint(0, 97, (1, 5), generator=torch.Generator().manual_seed(10 + rank))
    eng.eval()
    out = eng.generate(prompt, max_new_tokens=5)
    assert torch.equal(out, _greedy_ref(ref, prompt, 5))
    eng.train()
    x = torch.randint(0, 97, (2, 12))
    loss = eng(x, labels=x)
    eng.backward(loss)
    eng.step()
    eng.eval()
    assert eng.last_latency_report is not None and "Generate time" in eng.last_latency_report


def test_hybrid_engine_tp_generate_gloo():
    run_distributed(_hybrid_tp, 2)


def test_decode_attention_device_lengths_reference():
    """decode_attention(lens=, window=) over a larger cache buffer equals attention over the sliced cache (the
    contract the HIP-graph decode step relies on)."""
    from hcache_deepspeed_amd.ops.decode_attention import decode_attention, decode_attention_ref
    g = torch.Generator().manual_seed(0)
    B, H, Hkv, S, D = 3, 4, 2, 20, 16
    q = torch.randn(B, H, D, generator=g)
    k = torch.randn(B, Hkv, S, D, generator=g)
    v = torch.randn(B, Hkv, S, D, generator=g)
    for n, win in ((7, 0), (13, 4), (20, 0)):
        lens = torch.full((B, ), n, dtype=torch.int32)
        lo = max(0, n - win) if win else 0
        ref = decode_attention_ref(q, k[:, :, lo:n], v[:, :, lo:n], 0.25)
        assert torch.allclose(decode_attention(q, k, v, 0.25, lens=lens, window=win), ref, atol=1e-5)
