"""Long-context training path (CPU numerics): the summed-residual block boundary and the sequence-chunked MLP.

* ``LlamaModel.summed_boundary`` / activation checkpointing: a block takes and returns the summed residual stream, so a
  checkpointed block saves ONE [tokens, hidden] input (h + residual) instead of two -- same loss and gradients;
* ``LlamaMLP.chunk_rows``: above that many tokens the MLP runs in sequence chunks recomputed per chunk in backward
  (parallel/fpdt.fpdt_gated_ffn) -- same loss and gradients;
* ``ckpt_offload`` under the host activation cache: exactly one saved tensor per block reaches the cache's pack hook.
"""
import pytest
import torch

from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, LlamaMLP, tiny


def _model():
    torch.manual_seed(0)
    return LlamaForCausalLM(tiny(num_hidden_layers=3, vocab_size=128, hidden_size=64, intermediate_size=96,
                                 num_attention_heads=4, num_key_value_heads=2, head_dim=16))


def _grads(m, x):
    m.zero_grad(set_to_none=True)
    loss = m(x, labels=x)
    loss.backward()
    return loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("mode", ["summed", "ckpt", "mlp_chunks", "summed_chunks"])
def test_long_context_paths_match_plain(mode, monkeypatch):
    m = _model()
    x = torch.randint(0, 128, (2, 24))
    ref_loss, ref = _grads(m, x)
    if mode in ("summed", "summed_chunks"):
        m.model.summed_boundary = True
    if mode == "ckpt":
        m.gradient_checkpointing_enable()
    if mode in ("mlp_chunks", "summed_chunks"):
        monkeypatch.setattr(LlamaMLP, "chunk_rows", 16)  # 48 tokens -> 3 chunks
        monkeypatch.setattr(LlamaMLP, "chunk_min_tokens", 0)
    loss, g = _grads(m, x)
    torch.testing.assert_close(loss, ref_loss, rtol=1e-6, atol=1e-6)
    for n in ref:
        torch.testing.assert_close(g[n], ref[n], rtol=1e-5, atol=1e-6, msg=n)


def test_ckpt_offload_saves_one_tensor_per_block():
    """The cache sets the summed boundary: the pack hook sees one [tokens, hidden] input per block (round 4: two)."""
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache
    m = _model()
    x = torch.randint(0, 128, (2, 24))
    ref_loss, ref = _grads(m, x)
    cache = HostActivationCache(torch.device("cpu"), ckpt_offload=True, stash_attention=False).attach(m)
    assert m.model.summed_boundary
    seen = []
    orig = cache._pack

    def pack(t):
        if isinstance(t, torch.Tensor) and cache.cur_layer >= 0 and t.dim() == 2 and t.shape == (48, 64) \
                and not t.is_leaf:
            seen.append(cache.cur_layer)
        return orig(t)

    cache._pack = pack
    m.zero_grad(set_to_none=True)
    with cache.forward_context():
        loss = m(x, labels=x)
    loss.backward()
    torch.testing.assert_close(loss.detach(), ref_loss)
    for n, p in m.named_parameters():
        torch.testing.assert_close(p.grad, ref[n], rtol=1e-5, atol=1e-6, msg=n)
    assert sorted(seen) == [0, 1, 2], seen


def _zero3_losses(rank, world, chunk_rows, summed):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models import llama
    llama.LlamaMLP.chunk_rows = chunk_rows
    llama.LlamaMLP.chunk_min_tokens = 0
    torch.manual_seed(0)
    with ds.zero.Init():
        m = LlamaForCausalLM(tiny(num_hidden_layers=2, vocab_size=97, hidden_size=32, intermediate_size=64,
                                  num_attention_heads=4, num_key_value_heads=2, head_dim=8))
    m.model.summed_boundary = summed
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": 3}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    g = torch.Generator().manual_seed(3 + rank)
    out = []
    for _ in range(3):
        b = torch.randint(0, 97, (2, 16), generator=g)
        loss = eng(b, labels=b)
        eng.backward(loss)
        eng.step()
        out.append(float(loss))
    return out


def _run_zero3(rank, world):
    base = _zero3_losses(rank, world, 0, False)
    chunked = _zero3_losses(rank, world, 8, True)  # 32 tokens -> 4 MLP chunks, summed boundary
    assert len(base) == 3
    for a, b in zip(base, chunked):
        assert abs(a - b) < 1e-4 * max(1.0, abs(a)), (base, chunked)


def test_zero3_chunked_mlp_and_summed_boundary_match():
    """ZeRO-3 world 2 (gloo): the chunked MLP's weight gradients reach the partitioned flat gradients through the
    post-accumulate hooks exactly like the unchunked layers' -- same loss trajectory."""
    from tests.dist_utils import run_distributed
    run_distributed(_run_zero3, 2)
