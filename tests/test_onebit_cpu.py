"""1-bit Adam / 0-1 Adam / 1-bit LAMB and the error-compensated compressed all-reduce on gloo (reference
tests/unit/runtime/half_precision/onebit/test_onebit.py and tests/onebit/test_nccl_backend.py strategies)."""
import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


def test_pack_unpack_signs():
    from hcache_deepspeed_amd.runtime.comm import pack_signs, unpack_signs
    x = torch.randn(64)
    p = pack_signs(x)
    assert p.dtype == torch.uint8 and p.numel() == 8
    assert torch.equal(unpack_signs(p), torch.where(x >= 0, 1.0, -1.0))


def _compressed(rank, world):
    from hcache_deepspeed_amd.runtime.comm.compressed import compressed_allreduce, padded_size
    n = padded_size(1000, world)
    werr = torch.zeros(n)
    serr = torch.zeros(n // world)
    g = torch.Generator().manual_seed(rank)
    acc_in = torch.zeros(n)
    acc_out = torch.zeros(n)
    outs = []
    for t in range(40):
        x = torch.randn(n, generator=g)
        xs = [torch.empty_like(x) for _ in range(world)]
        torch.distributed.all_gather(xs, x)
        acc_in += torch.stack(xs).mean(0)
        out = compressed_allreduce(x.clone(), werr, serr)
        acc_out += out
        outs.append(out)
    # identical result on every rank
    o = [torch.empty_like(outs[-1]) for _ in range(world)]
    torch.distributed.all_gather(o, outs[-1])
    assert all(torch.equal(o[0], t) for t in o)
    # error feedback: the accumulated output tracks the accumulated true mean (residual = current errors)
    rel = (acc_out - acc_in).norm() / acc_in.norm()
    assert rel < 0.25, rel


def test_compressed_allreduce_error_feedback():
    run_distributed(_compressed, 2)


def _onebit(rank, world, opt_type, extra):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.runtime.fp16.onebit import OnebitZeroOptimizer
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 4,
           "optimizer": {"type": opt_type, "params": dict({"lr": 3e-3}, **extra)},
           "zero_optimization": {"stage": 0}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    assert isinstance(eng.optimizer, OnebitZeroOptimizer)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 97, (4, 12), generator=g)  # same batch every step: loss must fall
    losses = []
    for _ in range(10):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    assert eng.optimizer.compressing
    assert losses[-1] < losses[0] - 0.3, losses
    # replicas stay bit-identical (the compressed all-reduce output is the same on every rank)
    flat = eng.optimizer.store.master.clone()
    allf = [torch.empty_like(flat) for _ in range(world)]
    torch.distributed.all_gather(allf, flat)
    assert torch.equal(allf[0], allf[1])


@pytest.mark.parametrize("opt_type,extra", [("OneBitAdam", {"freeze_step": 3}),
                                            ("ZeroOneAdam", {"var_freeze_step": 6, "var_update_scaler": 2}),
                                            ("OneBitLamb", {"freeze_step": 3})])
def test_onebit_optimizers_train(opt_type, extra):
    run_distributed(_onebit, 2, opt_type, extra)
