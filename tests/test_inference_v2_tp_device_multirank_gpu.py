"""The v2 ragged serving engine (HCache) with tensor parallelism TP = 2 on the HIP device path, both ranks on the one
MI355X of the test box (gloo rendezvous; RCCL refuses two ranks on one device; the row-parallel all-reduces take
the one-shot symmetric all-reduce). Ragged prefill, HCache evict / restore from hidden-state latents and decode on
each rank's half of the heads and MLP must reproduce the full model's logits in bf16."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.gpu


def _run(rank, world, d):
    from hcache_deepspeed_amd.inference.v2 import build_engine_from_model
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = dict(head_dim=128, hidden_size=256, intermediate_size=512, vocab_size=211, num_attention_heads=4,
               num_key_value_heads=2, num_hidden_layers=3)
    m = LlamaForCausalLM(tiny(**cfg)).to(device="cuda", dtype=torch.bfloat16).eval()
    eng = build_engine_from_model(m, {"latent_mode": "hidden", "dtype": "bf16", "tensor_parallel": {"tp_size": world},
                                      "state_manager": {"max_context": 1024, "kv_block_size": 64}},
                                  device=torch.device("cuda"), num_kv_blocks=64)
    assert eng._model.tp == world
    g = torch.Generator().manual_seed(1)
    p1 = torch.randint(0, 211, (70, ), generator=g)
    p2 = torch.randint(0, 211, (33, ), generator=g)
    cont = torch.randint(0, 211, (4, ), generator=g)
    with torch.no_grad():
        full1 = m(torch.cat([p1, cont]).cuda()[None]).float()
        full2 = m(p2.cuda()[None]).float()
    tol = 6e-2
    logits, lats = eng.put([1, 2], [p1, p2])
    assert torch.allclose(logits[0].float(), full1[69], atol=tol, rtol=tol)
    assert torch.allclose(logits[1].float(), full2[-1], atol=tol, rtol=tol)
    eng.evict(1)
    eng.restore_kv([1], [p1], [lats[0]])
    for j in range(cont.numel()):
        lg, _ = eng.put([1], [cont[j:j + 1]], capture_latents=False)
        assert torch.allclose(lg[0].float(), full1[70 + j], atol=tol, rtol=tol), j
    if world > 1:
        from hcache_deepspeed_amd.comm import symmetric
        assert sum(sm.calls["all_reduce"] for sm in symmetric._cache.values()) > 0
    torch.save({"ok": True}, os.path.join(d, f"r{rank}.pt"))


def test_v2_engine_tp2_device_path_matches_full_model(tmp_path):
    run_distributed(_run, 2, str(tmp_path))
    assert all(os.path.exists(tmp_path / f"r{r}.pt") for r in range(2))
