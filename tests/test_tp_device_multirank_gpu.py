"""Tensor parallelism (AutoTP = 2) on the HIP device path, both ranks on the one MI355X of the test box.

The two processes rendezvous over gloo (RCCL refuses two ranks on one device). The row-parallel forward
all-reduces are small (<= 256 KiB) and take the default one-shot symmetric-memory all-reduce over IPC-mapped
buffers of the other process (comm/symmetric.py); the backward all-reduces go through torch.distributed (gloo on
device tensors, staged through host memory where gloo refuses them). The sharded projections, the fused kernels
and the ZeRO-3 optimizer run on the GPU.

A world-2 TP run on the full batch must follow the world-1 run in loss within bf16 tolerance."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_device_multirank_gpu import CFG, _staged

pytestmark = pytest.mark.gpu


def _run(rank, world, d, steps=3):
    import hcache_deepspeed_amd as hds
    import hcache_deepspeed_amd.comm as hcomm
    from hcache_deepspeed_amd.comm import symmetric
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.cuda.set_device(0)
    for name in ("all_gather_into_tensor", "reduce_scatter_tensor"):
        setattr(hcomm, name, _staged(name))
        setattr(hcomm.comm, name, getattr(hcomm, name))
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**CFG))
    cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True}, "gradient_clipping": 1.0,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 3}}
    if world > 1:
        cfg["tensor_parallel"] = {"autotp_size": world}
    eng, _, _, _ = hds.initialize(model=m, config=cfg)
    if world > 1:
        attn = m.model.layers[0].self_attn
        assert attn.n_q == CFG["num_attention_heads"] // world
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(0, CFG["vocab_size"], (2, 128), generator=g).to(eng.device)  # one batch: the loss must fall
    losses = []
    for _ in range(steps):
        loss = eng(ids, labels=ids)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    if world > 1:
        calls = sum(sm.calls["all_reduce"] for sm in symmetric._cache.values())
        assert calls > 0, "the TP forward all-reduces did not take the symmetric one-shot path"
    if rank == 0:
        torch.save({"losses": losses}, os.path.join(d, f"tp{world}.pt"))


def test_autotp_device_path_world2_matches_world1(tmp_path):
    d = str(tmp_path)
    run_distributed(_run, 1, d)
    run_distributed(_run, 2, d)
    a = torch.load(os.path.join(d, "tp1.pt"), weights_only=True)["losses"]
    b = torch.load(os.path.join(d, "tp2.pt"), weights_only=True)["losses"]
    for la, lb in zip(a, b):
        assert abs(la - lb) <= 2e-2 * abs(la), (a, b)
    assert b[-1] < b[0]
