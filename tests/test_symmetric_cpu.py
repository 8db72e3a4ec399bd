"""Symmetric-memory collectives: CPU-side contract (the kernels themselves run in tests/test_symmetric_gpu.py).

On CPU tensors / gloo the TP all-reduce entry (``small_all_reduce``) must take the torch.distributed path with the
same result, ``compile.symmetric_memory`` must leave the ZeRO collectives on torch.distributed, and the training
trajectory must not change."""
import torch

from tests.dist_utils import run_distributed


def _run(rank, world):
    import torch.distributed as dist
    from hcache_deepspeed_amd.comm import symmetric
    assert not symmetric.supported(None)  # no GPU here
    x = torch.arange(16, dtype=torch.float32) * (rank + 1)
    out = symmetric.small_all_reduce(x.clone(), None, max_kb=64)
    assert torch.equal(out, torch.arange(16, dtype=torch.float32) * sum(r + 1 for r in range(world)))
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    losses = {}
    for sym in (False, True):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(vocab_size=97, hidden_size=32, intermediate_size=64, num_hidden_layers=2,
                                  num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64))
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}},
               "zero_optimization": {"stage": 3}, "compile": {"symmetric_memory": sym}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        if sym:
            eng.compile()
            assert getattr(eng.optimizer, "_symm", None) is None  # CPU: stays on torch.distributed
        g = torch.Generator().manual_seed(3 + rank)
        out = []
        for _ in range(3):
            b = torch.randint(0, 97, (2, 10), generator=g)
            loss = eng(b, labels=b)
            eng.backward(loss)
            eng.step()
            out.append(float(loss))
        losses[sym] = out
    assert losses[False] == losses[True]
    dist.barrier()


def test_symmetric_cpu_fallbacks():
    run_distributed(_run, 2)
