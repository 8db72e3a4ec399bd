"""FPDT (chunked Ulysses attention + chunked FFN / logits loss) against unchunked single-process references.

Reference test analogue: tests/unit/sequence_parallelism/test_ulysses.py (FPDT case compares the chunked layer
to a plain attention). Parity here: outputs and gradients of the chunked path equal the dense path.
"""
import pytest
import torch

from tests.dist_utils import run_distributed


def _qkv_ref(x, w, cos, sin, n_q, n_kv, D, S):
    from hcache_deepspeed_amd.ops.attention import qkv_attention
    T = x.shape[0]
    qkv = torch.nn.functional.linear(x, w).view(T, n_q + 2 * n_kv, D)
    return qkv_attention(qkv, n_q, n_kv, cos, sin, seq_len=S, causal=True).reshape(T, -1)


def test_fpdt_attention_single_rank_chunks():
    from hcache_deepspeed_amd.ops.rope import rope_tables
    from hcache_deepspeed_amd.parallel.fpdt import fpdt_attention
    torch.manual_seed(0)
    B, S, H, n_q, n_kv, D = 2, 48, 64, 4, 2, 16
    x = torch.randn(B * S, H, requires_grad=True)
    w = (torch.randn((n_q + 2 * n_kv) * D, H) * 0.1).requires_grad_(True)
    cos, sin = rope_tables(S, D)
    y0 = _qkv_ref(x, w, cos, sin, n_q, n_kv, D, S)
    g = torch.randn_like(y0)
    gx0, gw0 = torch.autograd.grad(y0, (x, w), g)
    for nc in (1, 3, 4):
        y = fpdt_attention(x, w, None, cos, sin, n_q, n_kv, D, None, B, nc)
        gx, gw = torch.autograd.grad(y, (x, w), g)
        assert torch.allclose(y, y0, atol=1e-5), nc
        assert torch.allclose(gx, gx0, atol=1e-4), nc
        assert torch.allclose(gw, gw0, atol=1e-4), nc


def test_fpdt_attention_replays_checkpoint_stash(monkeypatch):
    """Inside a checkpointed block with the attention stash, the recompute takes every segment's (o, lse) back
    instead of re-running the segment-pair attention; outputs and gradients are unchanged, and a no-grad forward
    gives the same output without filling the segment store."""
    from hcache_deepspeed_amd.ops import attention as A
    from hcache_deepspeed_amd.ops.rope import rope_tables
    from hcache_deepspeed_amd.parallel import fpdt as F
    from hcache_deepspeed_amd.runtime.activation_checkpointing.checkpointing import checkpoint_saved_inputs
    torch.manual_seed(0)
    B, S, H, n_q, n_kv, D, nc = 2, 48, 64, 4, 2, 16, 3
    x = torch.randn(B * S, H, requires_grad=True)
    w = (torch.randn((n_q + 2 * n_kv) * D, H) * 0.1).requires_grad_(True)
    cos, sin = rope_tables(S, D)

    def block(xx):
        return F.fpdt_attention(xx, w, None, cos, sin, n_q, n_kv, D, None, B, nc).square()

    y0 = block(x)
    g = torch.randn_like(y0)
    gx0, gw0 = torch.autograd.grad(y0, (x, w), g)
    calls = []
    real = F.attn_block_fwd
    monkeypatch.setattr(F, "attn_block_fwd", lambda *a: calls.append(1) or real(*a))
    puts = []
    real_put = F._HostChunks.put
    monkeypatch.setattr(F._HostChunks, "put", lambda self, k, t: puts.append(k) or real_put(self, k, t))
    y = checkpoint_saved_inputs(block, x, stash_attention=True)
    n_fwd = len(calls)
    assert n_fwd == nc * (nc + 1) // 2 and not puts  # the no-grad first pass: every pair once, nothing stored
    y.backward(g)  # the weight is closed over: its gradient accumulates in .grad (reentrant-style checkpoint)
    gx, gw = x.grad, w.grad
    assert len(calls) == n_fwd  # the recompute replayed the stash
    assert len([k for k in puts if k[0] != "do"]) == 5 * nc  # q, k, v, o, lse of every segment (recompute)
    torch.testing.assert_close(y, y0)
    torch.testing.assert_close(gx, gx0)
    torch.testing.assert_close(gw, gw0)
    assert A.AttnStash.mode is None
    with torch.no_grad():
        torch.testing.assert_close(block(x), y0.detach())


def test_chunked_ffn_and_logits_loss():
    from hcache_deepspeed_amd.parallel.fpdt import FPDT_FFN, FPDT_LogitsLoss, fpdt_gated_ffn
    torch.manual_seed(1)
    x = torch.randn(32, 16, requires_grad=True)
    w1, b1 = torch.randn(48, 16, requires_grad=True), torch.randn(48, requires_grad=True)
    w2, b2 = torch.randn(16, 48, requires_grad=True), torch.randn(16, requires_grad=True)
    y, _ = FPDT_FFN(x, w1, b1, w2, b2, True, chunk_size=8)
    y0 = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(x, w1, b1),
                                                             approximate="tanh"), w2, b2)
    g = torch.randn_like(y)
    a = torch.autograd.grad(y, (x, w1, b1, w2, b2), g)
    b = torch.autograd.grad(y0, (x, w1, b1, w2, b2), g)
    for u, v in zip(a, b):
        assert torch.allclose(u, v, atol=1e-4)
    wu, wd = torch.randn(64, 16, requires_grad=True), torch.randn(16, 32, requires_grad=True)
    y = fpdt_gated_ffn(x, wu, wd, 4)
    y0 = torch.nn.functional.linear(torch.nn.functional.silu(x @ wu[:32].t()) * (x @ wu[32:].t()), wd)
    assert torch.allclose(y, y0, atol=1e-4)
    a = torch.autograd.grad(y, (x, wu, wd), g)
    b = torch.autograd.grad(y0, (x, wu, wd), g)
    for u, v in zip(a, b):
        assert torch.allclose(u, v, atol=1e-3)
    V = 40
    wl = torch.randn(V, 16, requires_grad=True)
    lab = torch.randint(0, V, (32, ))
    lab[3] = -100
    loss = FPDT_LogitsLoss(x, lab, wl, None, num_chunks=4)
    ref = torch.nn.functional.cross_entropy(x @ wl.t(), lab, reduction="none", ignore_index=-100)
    assert torch.allclose(loss, ref, atol=1e-5)
    a = torch.autograd.grad(loss.sum(), (x, wl))
    b = torch.autograd.grad(ref.sum(), (x, wl))
    for u, v in zip(a, b):
        assert torch.allclose(u, v, atol=1e-4)


def _fpdt_model(rank, world):
    import torch.distributed as tdist
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.parallel.fpdt import FPDTInputConstruct, enable_fpdt
    torch.manual_seed(0)
    cfg = tiny(hidden_size=64, intermediate_size=128, num_attention_heads=4, num_key_value_heads=2, head_dim=16,
               num_hidden_layers=2, vocab_size=97)
    ref = LlamaForCausalLM(cfg)
    m = LlamaForCausalLM(cfg)
    m.load_state_dict(ref.state_dict())
    S, chunk = 64, 16  # 4 global chunks -> 2 per rank, 8-token local chunks
    ids = torch.randint(0, 97, (2, S), generator=torch.Generator().manual_seed(3))
    tgt = torch.roll(ids, -1, 1)
    h0 = ref.model(ids)  # [B*S, H]
    loss0 = torch.nn.functional.cross_entropy(torch.nn.functional.linear(h0, ref.lm_head.weight).float(),
                                              tgt.reshape(-1), reduction="none")
    loss0.sum().backward()
    group = tdist.new_group(list(range(world)))
    enable_fpdt(m, group, chunk, offload=False, ffn_chunks=2)
    ic = FPDTInputConstruct(ids, tgt, None, None, None, chunk, world, rank)
    lid, ltgt, _, _, _ = ic.generate()
    h = m.model(lid)
    loss = torch.nn.functional.cross_entropy(torch.nn.functional.linear(h, m.lm_head.weight).float(),
                                             ltgt.reshape(-1), reduction="none")
    idx = ic.indices()
    assert torch.allclose(loss.view(2, -1), loss0.view(2, S)[:, idx], atol=2e-4), (loss.view(2, -1) -
                                                                                  loss0.view(2, S)[:, idx]).abs().max()
    loss.sum().backward()
    for (n, p), (_, p0) in zip(m.named_parameters(), ref.named_parameters()):
        g = p.grad.clone()
        tdist.all_reduce(g, group=group)
        assert torch.allclose(g, p0.grad, atol=2e-3, rtol=1e-3), (n, (g - p0.grad).abs().max())


def test_fpdt_llama_sp2_matches_single():
    run_distributed(_fpdt_model, 2)


@pytest.mark.gpu
def test_fpdt_attention_gpu_offload():
    """HIP FA block kernels + pinned-host segment offload vs the dense fused-QKV attention."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hcache_deepspeed_amd.ops.rope import rope_tables
    from hcache_deepspeed_amd.parallel.fpdt import fpdt_attention
    torch.manual_seed(0)
    B, S, H, n_q, n_kv, D = 2, 1024, 512, 8, 2, 128
    dev = torch.device("cuda")
    x = (torch.randn(B * S, H, device=dev) * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn((n_q + 2 * n_kv) * D, H, device=dev) * 0.05).bfloat16().requires_grad_(True)
    cos, sin = rope_tables(S, D, device=dev)
    y0 = _qkv_ref(x, w, cos, sin, n_q, n_kv, D, S)
    g = torch.randn_like(y0)
    gx0, gw0 = torch.autograd.grad(y0, (x, w), g)
    y = fpdt_attention(x, w, None, cos, sin, n_q, n_kv, D, None, B, 4, offload=True)
    gx, gw = torch.autograd.grad(y, (x, w), g)
    torch.cuda.synchronize()

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    assert rel(y, y0) < 1e-2
    assert rel(gx, gx0) < 2e-2
    assert rel(gw, gw0) < 2e-2
