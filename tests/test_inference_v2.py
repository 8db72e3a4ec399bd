"""Ragged serving engine + HCache (put -> latents, restore_kv): consistency with the training model.

The reference has no test for restore_kv/latents; these pin its semantics: restoring the KV
cache from host latents and continuing decoding must give the same logits as never evicting.
Runs on CPU (torch reference ops) and, marked gpu, on the MI355X with the HIP paged kernels.
"""
import pytest
import torch

from hcache_deepspeed_amd.inference.v2 import build_engine_from_model
from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny


def _model(device, dtype, **kw):
    torch.manual_seed(0)
    cfg = dict(head_dim=128, hidden_size=256, intermediate_size=512, vocab_size=211, num_attention_heads=4,
               num_key_value_heads=2, num_hidden_layers=3)
    cfg.update(kw)
    m = LlamaForCausalLM(tiny(**cfg)).to(device=device, dtype=dtype).eval()
    return m


def _full_logits(m, ids):
    with torch.no_grad():
        return m(ids[None]).float()  # [T, V]


def _devices():
    devs = [("cpu", torch.float32)]
    return devs


def _run_consistency(device, dtype, latent_mode, tol, sync_latents=True):
    m = _model(device, dtype)
    eng = build_engine_from_model(m, {"latent_mode": latent_mode, "dtype": {torch.float32: "fp32",
                                                                          torch.bfloat16: "bf16"}[dtype],
                                      "state_manager": {"max_context": 1024, "kv_block_size": 64}},
                                  device=torch.device(device), num_kv_blocks=64)
    g = torch.Generator().manual_seed(1)
    p1 = torch.randint(0, 211, (70, ), generator=g)
    p2 = torch.randint(0, 211, (33, ), generator=g)
    cont = torch.randint(0, 211, (5, ), generator=g)
    full1 = _full_logits(m, torch.cat([p1, cont]).to(device))
    full2 = _full_logits(m, p2.to(device))
    # ragged prefill of two sequences
    logits, lats = eng.put([1, 2], [p1, p2], sync_latents=sync_latents)  # async: evict / restore_kv wait
    assert logits.shape == (2, 211)
    assert torch.allclose(logits[0].float(), full1[69], atol=tol, rtol=tol)
    assert torch.allclose(logits[1].float(), full2[-1], atol=tol, rtol=tol)
    L = m.config.num_hidden_layers
    assert lats[0].shape[0] == L and lats[0].shape[1] == 70
    # HCache: drop seq 1's KV, restore from latents, continue decoding
    eng.evict(1)
    blocks_before = eng.free_blocks
    eng.restore_kv([1, 2], [p1, p2], [lats[0], None])
    assert eng.free_blocks == blocks_before - 2
    for j in range(cont.numel()):
        lg, _ = eng.put([1], [cont[j:j + 1]], capture_latents=False)
        assert torch.allclose(lg[0].float(), full1[70 + j], atol=tol, rtol=tol), j
    # scheduling API
    tokens, blocks = eng.query(1, 100, 10)
    assert tokens > 0
    eng.flush(1)
    eng.flush(2)
    assert eng.free_blocks == 64


@pytest.mark.parametrize("latent_mode", ["hidden", "kv"])
def test_hcache_consistency_cpu(latent_mode):
    _run_consistency("cpu", torch.float32, latent_mode, 2e-4)
    _run_consistency("cpu", torch.float32, latent_mode, 2e-4, sync_latents=False)


@pytest.mark.gpu
@pytest.mark.parametrize("sync_latents", [True, False])
@pytest.mark.parametrize("latent_mode", ["hidden", "kv"])
def test_hcache_consistency_gpu(latent_mode, sync_latents):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_consistency("cuda", torch.bfloat16, latent_mode, 6e-2, sync_latents)


def _run_fp8_latents(device, dtype, mode="hidden_fp8"):
    """latent_mode="hidden_fp8": H + 4 bytes per token-layer (e4m3 + an fp32 scale per token), restore continues
    decoding with logits within 2e-2 (relative, norm-wise) of the bf16/fp32 hidden-state restore."""
    m = _model(device, dtype)
    qmode = mode
    g = torch.Generator().manual_seed(1)
    p1 = torch.randint(0, 211, (70, ), generator=g)
    cont = torch.randint(0, 211, (6, ), generator=g)
    outs = {}
    for mode in ("hidden", qmode):
        eng = build_engine_from_model(m, {"latent_mode": mode, "dtype": {torch.float32: "fp32",
                                                                        torch.bfloat16: "bf16"}[dtype],
                                          "state_manager": {"max_context": 1024, "kv_block_size": 64}},
                                      device=torch.device(device), num_kv_blocks=64)
        _, lats = eng.put([1], [p1])
        if mode == "hidden_fp8":
            assert lats[0].dtype == torch.uint8 and lats[0].shape == (3, 70, 256 + 4)
        if mode == "hidden_int8":
            assert lats[0].dtype == torch.uint8 and lats[0].shape == (3, 70, 256 + 8)
        eng.evict(1)
        eng.restore_kv([1], [p1], [lats[0]])
        seq = []
        for j in range(cont.numel()):
            lg, _ = eng.put([1], [cont[j:j + 1]], capture_latents=False)
            seq.append(lg[0].float())
        outs[mode] = torch.stack(seq)
        eng.flush(1)
    a, b = outs["hidden"], outs[qmode]
    rel = ((a - b).norm(dim=-1) / a.norm(dim=-1)).max().item()
    assert rel < 2e-2, rel
    # greedy tokens agree wherever the reference's top-1 margin exceeds what the quantization moved the logits by
    # (on the random tiny model some steps are near-ties, which any lossy latent may flip)
    top2 = a.topk(2, dim=-1).values
    decided = (top2[:, 0] - top2[:, 1]) > 2 * (a - b).abs().max(dim=-1).values
    assert decided.any()
    assert torch.equal(a.argmax(-1)[decided], b.argmax(-1)[decided])


@pytest.mark.parametrize("mode", ["hidden_fp8", "hidden_int8"])
def test_hcache_quantized_latents_cpu(mode):
    _run_fp8_latents("cpu", torch.float32, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["hidden_fp8", "hidden_int8"])
def test_hcache_quantized_latents_gpu(mode):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_fp8_latents("cuda", torch.bfloat16, mode)


def test_hcache_auto_latent_mode_picks_smaller_lossless():
    m = _model("cpu", torch.float32)  # H = 256 < 2 x 2 kv heads x 128 = 512: the hidden state is smaller
    eng = build_engine_from_model(m, {"latent_mode": "auto", "dtype": "fp32",
                                      "state_manager": {"max_context": 256, "kv_block_size": 64}},
                                  device=torch.device("cpu"), num_kv_blocks=8)
    assert eng._model.latent_mode == "hidden"
    m2 = _model("cpu", torch.float32, hidden_size=1024, num_attention_heads=8, num_key_value_heads=2)
    eng2 = build_engine_from_model(m2, {"latent_mode": "auto", "dtype": "fp32",
                                        "state_manager": {"max_context": 256, "kv_block_size": 64}},
                                   device=torch.device("cpu"), num_kv_blocks=8)
    assert eng2._model.latent_mode == "kv"  # 2 x 2 x 128 = 512 < 1024


@pytest.mark.gpu
def test_decode_graph_matches_eager_gpu():
    """HIP-graph decode (one captured forward per batch size, replayed with new metadata) produces the logits of the
    eager ragged forward, across steps whose context lengths, KV slots and sequence sets change."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = _model("cuda", torch.bfloat16)
    econf = {"dtype": "bf16", "state_manager": {"max_context": 1024, "kv_block_size": 64}}
    engs = {}
    for mode in ("graph", "eager"):
        eng = build_engine_from_model(m, econf, device=torch.device("cuda"), num_kv_blocks=64)
        if mode == "eager":
            eng._model.decode_graph_max_batch = 0
        engs[mode] = eng
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, 211, (n, ), generator=g) for n in (40, 65, 7)]
    for eng in engs.values():
        eng.put([1, 2, 3], prompts, capture_latents=False)
    for step in range(6):
        uids = [1, 2, 3] if step % 3 else [1, 3]  # two batch sizes -> two captured graphs
        toks = [torch.randint(0, 211, (1, ), generator=g) for _ in uids]
        out = {k: e.put(uids, toks, capture_latents=False)[0].float() for k, e in engs.items()}
        assert torch.allclose(out["graph"], out["eager"], atol=2e-2, rtol=2e-2), step
    assert set(engs["graph"]._model._decode_graphs) == {(2, False), (3, False)}
    assert not engs["eager"]._model._decode_graphs


@pytest.mark.gpu
@pytest.mark.parametrize("latent_mode", ["kv", "hidden", "hidden_fp8"])
def test_graph_decode_captures_latents_for_restore_gpu(latent_mode):
    """HCache during HIP-graph decode: 64 graph-decoded tokens capture their latents into the device ring (drained in
    bulk, no per-token synchronize); evicting the sequence, restoring its KV from the prefill + decode latents and
    continuing gives the tokens of the uninterrupted run (kv: bit-exact K|V; hidden modes: logits within tolerance,
    tokens equal wherever the top-1 margin is decisive)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = _model("cuda", torch.bfloat16)
    econf = {"dtype": "bf16", "latent_mode": latent_mode, "state_manager": {"max_context": 1024, "kv_block_size": 64}}
    ref = build_engine_from_model(m, econf, device=torch.device("cuda"), num_kv_blocks=64)
    eng = build_engine_from_model(m, econf, device=torch.device("cuda"), num_kv_blocks=64)
    eng._model.decode_latent_ring_steps = 16
    g = torch.Generator().manual_seed(5)
    prompt = torch.randint(0, 211, (40, ), generator=g)
    lr, _ = ref.put([1], [prompt], capture_latents=False)
    le, lat0 = eng.put([1], [prompt])  # eager prefill: latents synchronized
    tr, te = lr.argmax(-1).cpu(), le.argmax(-1).cpu()
    fed, steps = [prompt], []
    for j in range(64):
        assert torch.equal(tr, te), j  # the capturing graph computes exactly what the plain graph computes
        fed.append(te.clone())
        lr, _ = ref.put([1], [tr], capture_latents=False)
        le, lat = eng.put([1], [te], sync_latents=False)  # graph decode, latents deferred to the ring
        steps.append(lat[0])
        tr, te = lr.argmax(-1).cpu(), le.argmax(-1).cpu()
    assert (1, True) in eng._model._decode_graphs and (1, False) in ref._model._decode_graphs
    assert not eng.latents_ready() or True  # (may already be drained: 64 = 4 full halves)
    eng.evict(1)  # waits for (and flushes) the ring
    assert eng.latents_ready()
    lat_all = torch.cat([lat0[0]] + steps, dim=1)
    assert lat_all.shape[:2] == (3, 40 + 64)
    eng.restore_kv([1], [torch.cat(fed)], [lat_all])
    outs = {"ref": [], "eng": []}
    for j in range(16):
        lr, _ = ref.put([1], [tr], capture_latents=False)
        le, _ = eng.put([1], [tr], capture_latents=False)  # same inputs: compare the continuations' logits
        outs["ref"].append(lr[0].float())
        outs["eng"].append(le[0].float())
        tr = lr.argmax(-1).cpu()
    a, b = torch.stack(outs["ref"]), torch.stack(outs["eng"])
    if latent_mode == "kv":
        assert torch.equal(a.argmax(-1), b.argmax(-1))
        assert torch.allclose(a, b, atol=1e-2, rtol=1e-2)
    else:
        rel = ((a - b).norm(dim=-1) / a.norm(dim=-1)).max().item()
        assert rel < (6e-2 if latent_mode == "hidden" else 1e-1), rel
        top2 = a.topk(2, dim=-1).values
        decided = (top2[:, 0] - top2[:, 1]) > 2 * (a - b).abs().max(dim=-1).values
        assert torch.equal(a.argmax(-1)[decided], b.argmax(-1)[decided])


def test_allocator_and_scheduling():
    from hcache_deepspeed_amd.inference.v2 import BlockedAllocator, SchedulingResult
    a = BlockedAllocator(10)
    x = a.allocate(4)
    assert a.free_blocks == 6
    a.free(x)
    assert a.free_blocks == 10
    with pytest.raises(ValueError):
        a.allocate(11)
    with pytest.raises(ValueError):
        a.free([3])
    m = _model("cpu", torch.float32, num_hidden_layers=1)
    eng = build_engine_from_model(m, {"dtype": "fp32", "state_manager": {"max_context": 256,
                                                                        "max_ragged_batch_size": 100}},
                                  device=torch.device("cpu"), num_kv_blocks=3)
    assert eng.can_schedule([1], [101]) == SchedulingResult.BatchTokenLimitExceeded
    assert eng.can_schedule([1], [300]) in (SchedulingResult.SequenceTokenLimitExceeded,
                                            SchedulingResult.BatchTokenLimitExceeded)
    assert eng.can_schedule([1, 2], [99, 1]) == SchedulingResult.Success
    assert eng.can_schedule([1], [64 * 3 + 1]) != SchedulingResult.Success


def test_native_ragged_metadata_matches_python_reference():
    """csrc/host/ragged_meta.cpp packs seq_meta / token maps / last rows / block tables / atoms exactly as the
    Python reference (ops/paged.build_atoms and the per-sequence loops) would build them."""
    import ctypes
    import numpy as np
    from hcache_deepspeed_amd.ops import native
    from hcache_deepspeed_amd.ops.paged import build_atoms
    lib = native.host_lib()
    rng = np.random.default_rng(0)
    n_q, n_kv, rpa, mb = 32, 8, 128, 6
    for S in (0, 1, 5):
        n_new = rng.integers(1, 70, S).astype(np.int32)
        seen = rng.integers(0, 200, S).astype(np.int32)
        blocks = [list(rng.integers(0, 1000, rng.integers(1, mb + 1))) for _ in range(S)]
        off = np.zeros(S + 1, dtype=np.int64)
        if S:
            off[1:] = np.cumsum([len(b) for b in blocks])
        flat = np.array([b for bl in blocks for b in bl], dtype=np.int32)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        need = ctypes.c_int64(0)
        out = np.zeros(1 << 16, dtype=np.int32)
        A = lib.hds_ragged_meta_build(P(n_new), P(seen), S, P(flat), P(off), mb, n_q, n_kv, rpa, P(out),
                                      out.size, ctypes.byref(need))
        meta_host = []
        q0 = 0
        for i in range(S):
            meta_host.append((q0, int(n_new[i]), int(seen[i])))
            q0 += int(n_new[i])
        T = q0
        ref_atoms, nref = build_atoms(meta_host, n_q, n_kv)
        assert A == nref and need.value == 4 * S + 2 * T + S * mb + 3 * A
        o = 0
        meta = out[o:o + 3 * S].reshape(S, 3); o += 3 * S
        tok_seq = out[o:o + T]; o += T
        tok_pos = out[o:o + T]; o += T
        last = out[o:o + S]; o += S
        tables = out[o:o + S * mb].reshape(S, mb); o += S * mb
        atoms = out[o:o + 3 * A].reshape(A, 3)
        assert meta.tolist() == [list(m) for m in meta_host]
        for i, (q, n, sn) in enumerate(meta_host):
            assert (tok_seq[q:q + n] == i).all() and tok_pos[q:q + n].tolist() == list(range(sn, sn + n))
            assert last[i] == q + n - 1
            assert tables[i, :len(blocks[i])].tolist() == blocks[i] and (tables[i, len(blocks[i]):] == 0).all()
        if A:
            assert atoms.tolist() == ref_atoms.tolist()


@pytest.mark.parametrize("latent_mode", ["hidden", "kv"])
def test_fused_decode_flow_cpu(latent_mode, monkeypatch):
    """The decode flow with the pre-norms and SwiGLU folded into the projection GEMVs (model._fused_decode_ok;
    off the GPU ops/gemv.fused_gemv runs the same arithmetic in torch): logits, evict / restore and the decode
    step's HCache latents match the unfused flow."""
    from hcache_deepspeed_amd.inference.v2.model import RaggedTransformer
    real = RaggedTransformer._fused_decode_ok
    _run_consistency("cpu", torch.float32, latent_mode, 2e-4)  # unfused, for the record
    monkeypatch.setattr(RaggedTransformer, "_fused_decode_ok", lambda self, T: T <= 2)
    _run_consistency("cpu", torch.float32, latent_mode, 2e-4)
    outs = []
    for fused in (False, True):
        monkeypatch.setattr(RaggedTransformer, "_fused_decode_ok", (lambda self, T: T <= 2) if fused else real)
        m = _model("cpu", torch.float32)
        eng = build_engine_from_model(m, {"latent_mode": latent_mode, "dtype": "fp32",
                                          "state_manager": {"max_context": 256, "kv_block_size": 64}},
                                      device=torch.device("cpu"), num_kv_blocks=16)
        g = torch.Generator().manual_seed(2)
        eng.put([1, 2], [torch.randint(0, 211, (20, ), generator=g), torch.randint(0, 211, (9, ), generator=g)])
        lg, lats = eng.put([1, 2], [torch.tensor([5]), torch.tensor([7])])  # a 2-row decode step, latents on
        outs.append((lg.float(), [l.float() for l in lats]))
    torch.testing.assert_close(outs[0][0], outs[1][0], atol=2e-4, rtol=2e-4)
    for a, b in zip(outs[0][1], outs[1][1]):
        torch.testing.assert_close(a, b, atol=2e-4, rtol=2e-4)
