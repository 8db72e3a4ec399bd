"""Coalesced / quantized gradient collectives, comm debug switches and muP optimizers on gloo
(reference tests/unit/comm/test_coalesced_collectives.py: reduce_scatter_coalesced on single/padded/multiple
tensors against the plain average; qgZ correctness within quantization tolerance)."""
import pytest
import torch

from tests.dist_utils import run_distributed


def _rs_coalesced(rank, world):
    from hcache_deepspeed_amd.runtime.comm.coalesced_collectives import reduce_scatter_coalesced
    shapes = [(8, ), (5, 3), (7, ), (world * 4, )]
    ts = [torch.arange(torch.Size(s).numel(), dtype=torch.float32).reshape(s) * (rank + 1) for s in shapes]
    outs = reduce_scatter_coalesced(ts)
    scale = sum(r + 1 for r in range(world)) / world
    for t, o in zip(ts, outs):
        full = torch.arange(t.numel(), dtype=torch.float32) * scale
        c = -(-t.numel() // world)
        ref = full[rank * c:(rank + 1) * c]
        assert o.numel() == ref.numel()
        torch.testing.assert_close(o, ref)


def _qgz(rank, world, hier):
    import hcache_deepspeed_amd.comm as dist
    from hcache_deepspeed_amd.runtime.comm import coalesced_collectives as cc
    groups = cc.create_qgz_groups(2) if hier else None
    g = torch.Generator().manual_seed(100 + rank)
    ts = [torch.randn(world * 16, 64, generator=g), torch.randn(world * 3, generator=g)]
    outs = cc.all_to_all_quant_reduce(ts, groups, bits=8)
    for t, o in zip(ts, outs):
        allt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        avg = torch.stack(allt).mean(0).reshape(-1)
        c = t.numel() // world
        ref = avg[rank * c:(rank + 1) * c]
        torch.testing.assert_close(o, ref, atol=0.05, rtol=0.05)
    # LoCo: error feedback keeps the running average closer to exact than plain quantization
    p = torch.nn.Parameter(torch.zeros(world * 16, 64))
    p.grad = ts[0].clone()
    acc = torch.zeros(p.numel() // world)
    for _ in range(4):
        acc += cc.all_to_all_loco_quant_reduce([p], groups, {"err_beta": 1.0, "reset_T": 100}, bits=4)[0]
    allt = [torch.empty_like(ts[0]) for _ in range(world)]
    dist.all_gather(allt, ts[0])
    c = p.numel() // world
    ref = torch.stack(allt).mean(0).reshape(-1)[rank * c:(rank + 1) * c] * 4
    assert (acc - ref).abs().max() < 0.5


def _switches(rank, world):
    import hcache_deepspeed_amd.comm as dist
    x = torch.full((4, ), float(rank + 1))
    dist.all_reduce_comm_off(True)
    dist.all_reduce(x)
    assert torch.all(x == rank + 1)
    dist.all_reduce_comm_off(False)
    dist.all_reduce(x)
    assert torch.all(x == sum(range(1, world + 1)))
    dist.backward_comm_off(True)
    out = torch.zeros(4 * world)
    dist.all_gather_into_tensor(out, torch.ones(4))
    assert torch.all(out == 0)
    dist.backward_comm_off(False)
    ins = [torch.full((3, ), float(rank)), torch.full((2, 2), 10.0 + rank)]
    outs = [torch.empty(3 * world), torch.empty(world * 2, 2)]
    dist.all_gather_coalesced(outs, ins)
    assert torch.equal(outs[0], torch.arange(world).float().repeat_interleave(3))
    assert torch.equal(outs[1].view(world, 4)[:, 0], 10.0 + torch.arange(world).float())
    assert dist.get_all_ranks_from_group() == list(range(world))
    with dist.coalescing_manager():
        pass


def test_reduce_scatter_coalesced():
    run_distributed(_rs_coalesced, 3)


@pytest.mark.parametrize("hier", [False, True])
def test_qgz_all_to_all_quant_reduce(hier):
    run_distributed(_qgz, 4, hier)


def test_comm_switches_and_coalesced_gather():
    run_distributed(_switches, 2)


def test_mup_optimizers():
    from hcache_deepspeed_amd.ops.mup import MuAdam, MuAdamW, MuSGD, set_base_shapes

    def mk(w):
        return torch.nn.Sequential(torch.nn.Linear(8, w), torch.nn.Linear(w, w), torch.nn.Linear(w, 4))

    base, model = mk(16), mk(64)
    set_base_shapes(model, base)
    hidden = model[1].weight
    assert hidden.mup_ninf == 2 and hidden.mup_width_mult == 4.0
    opt = MuAdamW(model.parameters(), lr=0.1, weight_decay=0.0)
    mults = {id(p): g["lr_mult"] for g in opt.param_groups for p in g["params"]}
    assert mults[id(hidden)] == pytest.approx(0.25)
    assert mults[id(model[0].bias)] == 1.0
    # the update of the hidden matrix is 1/width_mult of plain Adam's (first Adam step moves by ~lr)
    for p in model.parameters():
        p.grad = torch.ones_like(p)
    before = hidden.detach().clone()
    opt.step()
    assert (before - hidden.detach()).abs().max().item() == pytest.approx(0.1 / 4, rel=1e-3)
    # schedulers write the unscaled lr; the ratio survives
    for g in opt.param_groups:
        g["lr"] = 0.2
    before = hidden.detach().clone()
    opt.step()
    assert (before - hidden.detach()).abs().max().item() == pytest.approx(0.2 / 4, rel=0.05)
    s = MuSGD(model.parameters(), lr=0.1)
    assert any(g["lr_mult"] != 1.0 for g in s.param_groups)
    s.step()
    assert all(g["lr"] == 0.1 for g in s.param_groups)
    MuAdam(model.parameters(), lr=0.1, weight_decay=0.01).step()


def _mup_engine(rank, world):
    import hcache_deepspeed_amd as ds
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 16))
    for p in m.parameters():
        p.mup_width_mult = 2.0
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "MuAdamW", "params": {"lr": 1e-2}},
           "zero_optimization": {"stage": 2}}
    eng, opt, _, _ = ds.initialize(model=m, config=cfg)
    x = torch.randn(2, 16)
    for _ in range(2):
        loss = eng(x).pow(2).mean()
        eng.backward(loss)
        eng.step()
    assert any(g.get("lr_mult", 1.0) == 0.5 for g in eng.optimizer.param_groups)


def test_mup_through_engine_zero2():
    run_distributed(_mup_engine, 2)
