"""Ulysses sequence parallelism (SP = 2) on the HIP device path, both ranks on the one MI355X of the test box.

The ranks rendezvous over gloo (RCCL refuses two ranks on one device) and the head <-> sequence all-to-alls are
staged through host memory; the sharded attention (FlashAttention on each rank's heads over the full sequence), the
fused kernels and the optimizer run on the GPU. Each rank trains on its half of every sequence; the mean loss must
follow a world-1 run on the whole sequences within bf16 tolerance."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_moe_device_multirank_gpu import _staged_all_to_all
from tests.test_zero_device_multirank_gpu import CFG, _staged

pytestmark = pytest.mark.gpu

S = 256


def _run(rank, world, d, steps=3, extra=None, tag=""):
    import hcache_deepspeed_amd as hds
    import hcache_deepspeed_amd.comm as hcomm
    import torch.distributed as tdist
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.cuda.set_device(0)
    for name in ("all_gather_into_tensor", "reduce_scatter_tensor"):
        setattr(hcomm, name, _staged(name))
        setattr(hcomm.comm, name, getattr(hcomm, name))
    hcomm.all_to_all_single = _staged_all_to_all()
    hcomm.comm.all_to_all_single = hcomm.all_to_all_single
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**CFG))
    cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True}, "gradient_clipping": 1.0,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 1}}
    if world > 1:
        cfg["sequence_parallel_size"] = world
    if extra:
        cfg["mi355x"] = dict(extra)
    eng, _, _, _ = hds.initialize(model=m, config=cfg)
    g = torch.Generator().manual_seed(11)
    x = torch.randint(0, CFG["vocab_size"], (2, S + 1), generator=g)
    x, t = x[:, :-1].contiguous(), x[:, 1:].contiguous()
    idx = eng.sequence_shard_indices(S)  # contiguous slice (Ulysses) or the FPDT chunk layout
    xs = x[:, idx].contiguous().to(eng.device)
    ts = t[:, idx].contiguous().to(eng.device)
    losses = []
    for _ in range(steps):
        loss = eng(xs, targets=ts)
        eng.backward(loss)
        eng.step()
        lt = loss.detach().float().cpu()
        if world > 1:
            tdist.all_reduce(lt)
        losses.append(float(lt) / world)
    ac = getattr(eng, "_activation_cache", None)
    if rank == 0:
        torch.save({"losses": losses, "offloaded": ac.stats()["bytes_offloaded"] if ac is not None else 0},
                   os.path.join(d, f"sp{world}{tag}.pt"))


def test_ulysses_device_path_world2_matches_world1(tmp_path):
    d = str(tmp_path)
    run_distributed(_run, 1, d)
    run_distributed(_run, 2, d)
    a = torch.load(os.path.join(d, "sp1.pt"), weights_only=True)["losses"]
    b = torch.load(os.path.join(d, "sp2.pt"), weights_only=True)["losses"]
    for la, lb in zip(a, b):
        assert abs(la - lb) <= 2e-2 * abs(la), (a, b)
    assert b[-1] < b[0]


@pytest.mark.parametrize("mode", ["ckpt_offload", "fpdt+ckpt_offload"])
def test_ulysses_long_context_stack_world2_matches_world1(tmp_path, mode):
    """SP = 2 with the host activation cache (ckpt_offload: every block checkpointed, its boundary spilled to pinned
    host memory and prefetched back) and optionally FPDT attention (segments offloaded between forward and backward),
    both ranks on the one MI355X: losses follow the world-1 run on whole sequences (VERDICT r5 Next 2)."""
    d = str(tmp_path)
    extra = {"host_act_cache": {"enabled": True, "policy": "ckpt_offload", "min_kib": 16}}
    if mode.startswith("fpdt"):
        extra["fpdt"] = {"enabled": True, "chunk_size": 64, "offload": True}
    run_distributed(_run, 1, d)
    run_distributed(_run, 2, d, 3, extra, "_" + mode)
    a = torch.load(os.path.join(d, "sp1.pt"), weights_only=True)["losses"]
    rec = torch.load(os.path.join(d, f"sp2_{mode}.pt"), weights_only=True)
    b = rec["losses"]
    for la, lb in zip(a, b):
        assert abs(la - lb) <= 2e-2 * abs(la), (a, b)
    assert rec["offloaded"] > 0  # boundaries really went to the host
