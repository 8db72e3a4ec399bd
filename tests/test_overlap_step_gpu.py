"""Overlapped ZeRO-3 step on the GPU (runtime/zero/optimizer.py ``_overlap_ok`` / ``_step_pieces``): the fused Adam
runs unit by unit on a side stream after ``step()`` returns, each unit's forward waits for its own piece. The
trajectory must follow the synchronous step (the same kernel over the same elements, split by unit) within the
run-to-run noise of the synchronous step itself, with no host synchronisation inside the loop to hide a missing
wait."""
import os

import pytest
import torch


def _run(overlap, steps=5, tied=False):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.utils.tensor_fragment import safe_get_full_fp32_param
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(hidden_size=256, intermediate_size=512, num_hidden_layers=4, num_attention_heads=2,
                              num_key_value_heads=1, vocab_size=512, tie_word_embeddings=tied))
    # lr 1e-2: a forward that read a unit one update late would move the weights visibly
    cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True}, "gradient_clipping": 1.0,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}},
           "zero_optimization": {"stage": 3}, "mi355x": {"overlap_step": overlap}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    init = {n: safe_get_full_fp32_param(p).float().cpu() for n, p in eng.module.named_parameters()}
    g = torch.Generator(device="cuda").manual_seed(5)
    losses = []
    for _ in range(steps):
        x = torch.randint(0, 512, (2, 128), device="cuda", generator=g)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(loss.detach())  # no .item() in the loop: nothing syncs the host with the side stream
    eng._settle_host_step()  # what checkpoints / state dicts do first: the last overlapped step is complete
    out = {n: safe_get_full_fp32_param(p).float().cpu() for n, p in eng.module.named_parameters()}
    torch.cuda.synchronize()
    n = getattr(eng.optimizer, "overlapped_steps", 0)
    return torch.stack(losses).float().cpu(), init, out, n


@pytest.mark.gpu
@pytest.mark.parametrize("tied", [False, True])
def test_overlapped_step_matches_synchronous(tied):
    """The overlapped run must follow the synchronous one: per tensor, the mean |difference| of the fp32 masters
    stays a small fraction of how far five steps moved them. Float-atomic reductions (global norm, norm-weight
    gradients) make any two runs differ a little; a forward that read a unit before its update landed would be off
    by a whole update on every element of that unit."""
    os.environ.setdefault("MASTER_PORT", "29571")
    la, init, pa, n0 = _run(False, tied=tied)
    l1, _, p1, n1 = _run(True, tied=tied)
    assert n0 == 0 and n1 == 5
    assert torch.equal(la[:1], l1[:1])  # the first forward precedes any update
    assert (l1 - la).abs().max().item() <= 0.05 * (la[0] - la[-1]).abs().item() + 1e-3, (la, l1)
    assert pa.keys() == p1.keys()
    for k in pa:
        moved = (pa[k] - init[k]).abs().mean().item()
        diff = (p1[k] - pa[k]).abs().mean().item()
        assert diff <= 0.05 * moved + 1e-7, (k, diff, moved)
