"""GPT-2 small geometry (head_dim 64) on the GPU: every attention call is the HIP FlashAttention kernel (the
SDPA fallback is disabled), and bf16 forward/backward tracks the fp32 CPU model on the same weights."""
import pytest
import torch


@pytest.mark.gpu
def test_gpt2_small_heads_hip_attention(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hcache_deepspeed_amd.models import gpt2 as G
    torch.manual_seed(0)
    cfg = G.GPT2Config(vocab_size=1000, n_positions=512, n_embd=768, n_layer=2, n_head=12)
    ref = G.GPT2LMHeadModel(cfg).float()
    gpu = G.GPT2LMHeadModel(cfg)
    gpu.load_state_dict(ref.state_dict())
    gpu = gpu.cuda().to(torch.bfloat16)
    x = torch.randint(0, cfg.vocab_size, (2, 256))
    loss_ref = ref(x, labels=x)
    loss_ref.backward()

    def no_sdpa(*a, **k):
        raise AssertionError("SDPA ran instead of the HIP FlashAttention kernel")

    monkeypatch.setattr(G.F, "scaled_dot_product_attention", no_sdpa)
    loss = gpu(x.cuda(), labels=x.cuda())
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(loss_ref)) < 2e-2 * abs(float(loss_ref))
    for (n, a), (_, b) in zip(gpu.named_parameters(), ref.named_parameters()):
        if b.grad is None or "wpe" in n:
            continue
        rel = ((a.grad.float().cpu() - b.grad).norm() / (b.grad.norm() + 1e-12)).item()
        assert rel < 6e-2, (n, rel)
