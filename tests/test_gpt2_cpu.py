"""GPT-2: logits parity with HF transformers' GPT2LMHeadModel (converted weights) and the BASELINE plumbing config
"GPT-2-small ZeRO-1 on CPU + gloo world_size=2" (tiny width here; same code path) against plain torch AdamW."""
import pytest
import torch

from tests.dist_utils import run_distributed


def test_gpt2_matches_hf_logits():
    from transformers import GPT2Config as HFConfig, GPT2LMHeadModel as HFModel
    from hcache_deepspeed_amd.models.gpt2 import GPT2LMHeadModel, convert_hf_state_dict, gpt2_tiny
    torch.manual_seed(0)
    cfg = gpt2_tiny()
    hf = HFModel(HFConfig(vocab_size=cfg.vocab_size, n_positions=cfg.n_positions, n_embd=cfg.n_embd,
                          n_layer=cfg.n_layer, n_head=cfg.n_head, resid_pdrop=0, embd_pdrop=0, attn_pdrop=0)).eval()
    ours = GPT2LMHeadModel(cfg).eval()
    missing, unexpected = ours.load_state_dict(convert_hf_state_dict(hf.state_dict()), strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    x = torch.randint(0, cfg.vocab_size, (2, 16))
    with torch.no_grad():
        want = hf(x).logits
        got = ours(x)
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()
    # loss parity (HF shifts labels internally)
    with torch.no_grad():
        assert torch.allclose(ours(x, labels=x), hf(x, labels=x).loss, atol=1e-5)


def _zero1(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.gpt2 import GPT2LMHeadModel, gpt2_tiny
    torch.manual_seed(0)
    m = GPT2LMHeadModel(gpt2_tiny())
    ref = GPT2LMHeadModel(gpt2_tiny())
    ref.load_state_dict(m.state_dict())
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.0)
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3,
                                                                                          "weight_decay": 0.0}},
           "zero_optimization": {"stage": 1}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    g = torch.Generator().manual_seed(5)
    for _ in range(3):
        x = torch.randint(0, 256, (world * 2, 16), generator=g)
        loss = eng(x[rank * 2:(rank + 1) * 2], labels=x[rank * 2:(rank + 1) * 2])
        eng.backward(loss)
        eng.step()
        rl = ref(x, labels=x)
        rl.backward()
        opt.step()
        opt.zero_grad()
        tot = loss.detach().clone()
        torch.distributed.all_reduce(tot)
        assert float(tot) / world == pytest.approx(float(rl), rel=1e-4, abs=1e-4)


def test_gpt2_zero1_gloo_world2():
    run_distributed(_zero1, 2)
