"""Pipeline parallelism (1F1B) on the HIP device path, both stages on the one MI355X of the test box.

The stages rendezvous over gloo (RCCL refuses two ranks on one device) and the activation / gradient sends between
them are staged through host memory; the stage compute, the schedule's buffers and the optimizer run on the GPU.
Losses must follow single-process training of the same layer stack (the CPU test's reference) in fp32 -- this test
found the fused optimizers writing their bf16 parameter copy into fp32 training's compute buffer (ops/optimizers.py
``_native_lp``)."""
import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_pipe_cpu import V, _reference, _specs, loss_fn

pytestmark = pytest.mark.gpu


def _staged_batch_p2p(ops):
    import torch.distributed as tdist
    works, copies = [], []
    for kind, t, peer in ops:
        if kind == "send":
            works.append(tdist.isend(t.detach().contiguous().cpu(), peer))
        else:
            buf = torch.empty(t.shape, dtype=t.dtype)
            works.append(tdist.irecv(buf, peer))
            copies.append((t, buf))
    for w in works:
        w.wait()
    for t, buf in copies:
        t.copy_(buf)


def _pipe(rank, world, M):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.runtime.pipe import p2p
    from hcache_deepspeed_amd.runtime.pipe.engine import PipelineEngine
    from hcache_deepspeed_amd.runtime.pipe.module import PipelineModule
    torch.cuda.set_device(0)
    p2p.batch_p2p = _staged_batch_p2p
    mb, steps = 2, 3
    g = torch.Generator().manual_seed(3)
    glob = [torch.randint(0, V, (M * mb, 6), generator=g) for _ in range(steps)]
    glob = [(x, torch.roll(x, -1, dims=1)) for x in glob]
    ref = _reference(glob, steps, 1e-2)
    model = PipelineModule(_specs(), num_stages=world, loss_fn=loss_fn, seed_layers=True, base_seed=1234,
                           partition_method="parameters")
    cfg = {"train_micro_batch_size_per_gpu": mb, "gradient_accumulation_steps": M,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": 0}}
    eng, _, _, _ = ds.initialize(model=model, config=cfg)
    assert isinstance(eng, PipelineEngine) and eng.device.type == "cuda"
    assert all(p.is_cuda for p in eng.module.parameters())
    losses = []
    for x, y in glob:
        batches = [(a.cuda(), b.cuda()) for a, b in zip(x.split(mb), y.split(mb))]
        losses.append(float(eng.train_batch(iter(batches))))
    assert losses == pytest.approx(ref, rel=2e-3, abs=2e-3), (losses, ref)


@pytest.mark.parametrize("world,M", [(1, 2), (2, 4)])
def test_pipeline_device_path_matches_single_process(world, M):
    run_distributed(_pipe, world, M)
