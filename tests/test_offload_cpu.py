"""Host memory tier: CPU optimizers vs torch, async file I/O, ZeRO-Offload / NVMe-offload vs on-device ZeRO."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


def test_cpu_adam_matches_torch():
    from hcache_deepspeed_amd.ops.cpu_optimizers import DeepSpeedCPUAdam, cpu_adam_flat
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(10007))
    r = torch.nn.Parameter(p.detach().clone())
    opt = DeepSpeedCPUAdam([p], lr=1e-2, weight_decay=0.1)
    ropt = torch.optim.AdamW([r], lr=1e-2, weight_decay=0.1)
    for _ in range(4):
        g = torch.randn(10007)
        p.grad, r.grad = g, g.clone()
        opt.step()
        ropt.step()
    assert torch.allclose(p, r, atol=1e-6)
    # bf16 grads + bf16 param output
    p32 = torch.randn(4096)
    m, v = torch.zeros(4096), torch.zeros(4096)
    g = torch.randn(4096).to(torch.bfloat16)
    out = torch.empty(4096, dtype=torch.bfloat16)
    cpu_adam_flat(p32, g, m, v, 1, 1e-3, bf16_out=out)
    assert torch.equal(out, p32.to(torch.bfloat16))


def test_cpu_lion_adagrad_run():
    from hcache_deepspeed_amd.ops.cpu_optimizers import DeepSpeedCPUAdagrad, DeepSpeedCPULion
    for cls, ref in ((DeepSpeedCPUAdagrad, torch.optim.Adagrad), ):
        p = torch.nn.Parameter(torch.randn(1000))
        r = torch.nn.Parameter(p.detach().clone())
        o, ro = cls([p], lr=1e-2), ref([r], lr=1e-2)
        g = torch.randn(1000)
        p.grad, r.grad = g, g.clone()
        o.step()
        ro.step()
        assert torch.allclose(p, r, atol=1e-5)
    p = torch.nn.Parameter(torch.randn(1000))
    before = p.detach().clone()
    o = DeepSpeedCPULion([p], lr=1e-3)
    p.grad = torch.ones(1000)
    o.step()
    assert torch.allclose(p, before - 1e-3, atol=1e-6)


def test_aio_roundtrip(tmp_path):
    from hcache_deepspeed_amd.ops.aio import aio_handle
    h = aio_handle(block_size=1 << 16, intra_op_parallelism=3)
    t = torch.randn(1 << 18)
    f = str(tmp_path / "x.bin")
    h.sync_pwrite(t, f)
    u = torch.empty_like(t)
    h.sync_pread(u, f)
    assert torch.equal(t, u)
    # async with offsets
    a, b = torch.randn(1024), torch.randn(1024)
    h.async_pwrite(a, f, file_offset=0)
    h.async_pwrite(b, f, file_offset=4096)
    assert h.wait() == 2
    x, y = torch.empty(1024), torch.empty(1024)
    h.async_pread(x, f, 0)
    h.async_pread(y, f, 4096)
    h.wait()
    assert torch.equal(x, a) and torch.equal(y, b)


def _offload_vs_device(rank, world, stage, device, ratio, d, param=False):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    res = {}
    for mode in ("device", "offload"):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        z = {"stage": stage}
        if mode == "offload":
            z["offload_optimizer"] = {"device": device, "nvme_path": os.path.join(d, f"nvme{rank}"), "ratio": ratio}
            z["sub_group_size"] = 20000
            if param:
                z["offload_param"] = {"device": "cpu", "pin_memory": True}
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
               "zero_optimization": z, "gradient_clipping": 1.0}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        g = torch.Generator().manual_seed(10 + rank)
        for _ in range(3):
            x = torch.randint(0, 97, (2, 12), generator=g)
            loss = eng(x, labels=x)
            eng.backward(loss)
            eng.step()
        if param and mode == "offload":
            assert eng.optimizer.offload_param and eng.optimizer.store.lp.device.type == "cpu"
            assert eng.optimizer.partitioned
        res[mode] = eng.optimizer.full_fp32_state_dict(eng._param_names)
    for k in res["device"]:
        assert torch.allclose(res["device"][k], res["offload"][k], atol=1e-5), k


@pytest.mark.parametrize("stage,device,ratio", [(2, "cpu", 1.0), (3, "cpu", 1.0), (3, "nvme", 1.0),
                                                (2, "cpu", 0.5)])
def test_zero_offload_matches_device(stage, device, ratio, tmp_path):
    run_distributed(_offload_vs_device, 2, stage, device, ratio, str(tmp_path))


@pytest.mark.parametrize("world", [1, 2])
def test_zero_infinity_param_offload_matches_device(world, tmp_path):
    """ZeRO-Infinity: offload_param + offload_optimizer (cpu) reproduce the on-device ZeRO-3 trajectory."""
    run_distributed(_offload_vs_device, world, 3, "cpu", 1.0, str(tmp_path), True)


def test_act_cache_plan_spills_earliest_layers_within_budget():
    """Host activation cache budget planner: spill the shortest prefix of layers that fits the HBM budget."""
    from hcache_deepspeed_amd.offload.activation_cache import plan_offload
    lb = {i: 10 for i in range(8)}
    assert plan_offload(lb, peak_all=100, budget=1000) == set()          # everything fits: spill nothing
    assert plan_offload(lb, peak_all=100, budget=135) == set(range(5))   # 3 layers (30 B) fit next to the peak
    assert plan_offload(lb, peak_all=100, budget=99) == set(range(8))    # nothing fits: spill all
    assert plan_offload({}, peak_all=0, budget=1) == set()
