"""zero.Init semantics (reference runtime/zero/partition_parameters.py :302-615, :1108-1472; tests/unit/runtime/zero/
test_zero_context.py) and ZeRO-3 for models without ModuleLists (reference parameter_offload.py:281-460).

* parameters are partitioned as each module finishes __init__ (numel()==0, ds_shape/ds_numel kept);
* values written in __init__, loaded with load_state_dict inside the context, or modified under
  GatheredParameters(modifier_rank=0) survive into the engine;
* a model loaded inside zero.Init trains at world 2 on the same trajectory as unsharded torch AdamW;
* an nn.Sequential gets real ZeRO-3 sharding: empty parameters outside forward, the right answers;
* remote_device="cpu" keeps partitions in host memory.
"""
import pytest
import torch
import torch.nn as nn

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


class _ConstInit(nn.Module):

    def __init__(self):
        super().__init__()
        self.lin = nn.Linear(16, 8)
        with torch.no_grad():
            self.lin.weight.fill_(0.25)  # a value set in __init__ must survive partitioning
            self.lin.bias.copy_(torch.arange(8.0))

    def forward(self, x):
        return self.lin(x)


def _construct(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.runtime.zero.partition_parameters import gather_init_param
    with ds.zero.Init():
        m = LlamaForCausalLM(tiny(**TINY))
        c = _ConstInit()
    for n, p in m.named_parameters():
        assert p.numel() == 0, n
        assert p.ds_numel == torch.Size(p.ds_shape).numel()
        assert p._hds_part.numel() == -(-p.ds_numel // world)
    assert torch.equal(gather_init_param(c.lin.weight), torch.full((8, 16), 0.25))
    assert torch.equal(gather_init_param(c.lin.bias), torch.arange(8.0))
    with ds.zero.Init(remote_device="cpu"):
        r = nn.Linear(32, 32)
    assert r.weight._hds_part.device.type == "cpu"
    # GatheredParameters before initialize: rank 0's modification lands in every partition
    with ds.zero.GatheredParameters([c.lin.weight], modifier_rank=0):
        assert c.lin.weight.shape == (8, 16)
        if rank == 0:
            with torch.no_grad():
                c.lin.weight.fill_(-1.0)
    assert c.lin.weight.numel() == 0
    assert torch.equal(gather_init_param(c.lin.weight), torch.full((8, 16), -1.0))


def test_init_partitions_at_construction():
    run_distributed(_construct, 2)


def _loaded_trajectory(rank, world, stage):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    ref = LlamaForCausalLM(tiny(**TINY))
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    torch.manual_seed(1234 + rank)  # different default init per rank: only the loaded values may matter
    with ds.zero.Init():
        m = LlamaForCausalLM(tiny(**TINY))
        m.load_state_dict(sd)  # strict load inside the context
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3,
                                                                                           "weight_decay": 0.0}},
           "zero_optimization": {"stage": stage}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    for k, v in ref.state_dict().items():
        assert torch.equal(full[k], v), k
    ropt = torch.optim.AdamW(ref.parameters(), lr=5e-3, weight_decay=0.0)
    g = torch.Generator().manual_seed(5)
    for _ in range(3):
        b = torch.randint(0, 97, (2 * world, 12), generator=g)
        mine = b[2 * rank:2 * rank + 2]
        eng.backward(eng(mine, labels=mine))
        eng.step()
        ref(b, labels=b).backward()
        ropt.step()
        ropt.zero_grad()
    full = eng.optimizer.full_fp32_state_dict(eng._param_names)
    for n, p in ref.named_parameters():
        assert torch.allclose(full[n], p.detach(), atol=2e-5, rtol=1e-4), n


@pytest.mark.parametrize("stage", [3, 2])
def test_state_dict_loaded_inside_init_trains_like_unsharded(stage):
    run_distributed(_loaded_trajectory, 2, stage)


def _sequential(rank, world, use_init):
    import hcache_deepspeed_amd as ds
    torch.manual_seed(0)

    def net():
        return nn.Sequential(nn.Linear(32, 64), nn.GELU(), nn.Linear(64, 64), nn.GELU(), nn.Linear(64, 32),
                             nn.LayerNorm(32), nn.Linear(32, 4))

    ref = net()
    if use_init:
        with ds.zero.Init():
            m = net()
            m.load_state_dict(ref.state_dict())
    else:
        m = net()
        m.load_state_dict(ref.state_dict())
    cfg = {"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "AdamW", "params": {"lr": 1e-2,
                                                                                           "weight_decay": 0.0}},
           "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 100},
           "mi355x": {"zero3_unit_bucket_mb": 0.01}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    z = eng.optimizer
    fetch = [u for u in z.units if not u.persistent]
    assert len(fetch) >= 3, [(u.name, u.numel) for u in z.units]
    # LayerNorm params (32 < threshold) stay persistent, the Linears are sharded and empty outside forward
    assert m[5].weight.numel() == 32
    for i in (0, 2, 4, 6):
        assert m[i].weight.numel() == 0, i
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    g = torch.Generator().manual_seed(3)
    for _ in range(4):
        x = torch.randn(4 * world, 32, generator=g)
        y = torch.randn(4 * world, 4, generator=g)
        xm, ym = x[4 * rank:4 * rank + 4], y[4 * rank:4 * rank + 4]
        loss = ((eng(xm) - ym) ** 2).mean()
        eng.backward(loss)
        eng.step()
        ((ref(x) - y) ** 2).mean().backward()
        ropt.step()
        ropt.zero_grad()
        for i in (0, 2, 4, 6):
            assert m[i].weight.numel() == 0
    full = z.full_fp32_state_dict(eng._param_names)
    for n, p in ref.named_parameters():
        assert torch.allclose(full[n], p.detach(), atol=1e-5, rtol=1e-4), n


@pytest.mark.parametrize("use_init", [False, True])
def test_sequential_model_zero3_submodule_units(use_init):
    run_distributed(_sequential, 2, use_init)


def _external(rank, world):
    """A module whose forward reads another module's weight registers it as external: ZeRO-3 gathers it."""
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.runtime.zero import register_external_parameter

    class Tied(nn.Module):

        def __init__(self):
            super().__init__()
            self.a = nn.Linear(16, 16)
            self.b = nn.Linear(16, 16)
            self.head = _Head(self.a)

        def forward(self, x):
            return self.head(self.b(x))

    class _Head(nn.Module):

        def __init__(self, src):
            super().__init__()
            self.src = [src]  # not a submodule
            self.scale = nn.Parameter(torch.ones(16))
            register_external_parameter(self, src.weight)

        def forward(self, x):
            return (x @ self.src[0].weight.t()) * self.scale

    torch.manual_seed(0)
    ref = Tied()
    m = Tied()
    m.load_state_dict(ref.state_dict())
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "SGD", "params": {"lr": 0.1}},
           "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0},
           "mi355x": {"zero3_unit_bucket_mb": 0.0005}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    x = torch.randn(2, 16)
    out = eng(x)
    assert torch.allclose(out, ref(x), atol=1e-6)


def test_register_external_parameter_gathers_unit():
    run_distributed(_external, 2)
