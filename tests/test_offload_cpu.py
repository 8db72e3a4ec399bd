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


def test_act_cache_host_capped_calibration_plans_like_uncapped():
    """A calibration step whose pinned-host cap kept some layers on the GPU must plan the same spill set as an
    uncapped one: the capped bytes are inside the measured peak and must not be counted twice."""
    from hcache_deepspeed_amd.offload.activation_cache import calibrated_plan, plan_offload
    lb = {i: 10 for i in range(30)}
    base = 130  # model states + working set with every eligible layer on the host
    for budget in (140, 200, 265, 1000):
        uncapped = plan_offload(lb, peak_all=base, budget=budget)
        for capped_layers in (0, 5, 15):  # the cap kept the LAST layers of the forward on the GPU
            capped = capped_layers * 10
            assert calibrated_plan(lb, base + capped, capped, budget) == uncapped, (budget, capped_layers)


def _nvme_vs_dram(rank, world, d, opt_device, param_device):
    """ZeRO-Infinity NVMe tier: optimizer states (and parameters) in swap files reproduce the in-DRAM offload
    trajectory bit for bit; the swap files exist and carry the bytes (nothing silently stays in DRAM)."""
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    res = {}
    for mode in ("dram", "nvme"):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        path = os.path.join(d, f"{mode}{rank}")
        z = {"stage": 3, "sub_group_size": 7000,
             "offload_optimizer": {"device": "cpu" if mode == "dram" else opt_device, "nvme_path": path,
                                   "pin_memory": True},
             "offload_param": {"device": "cpu" if mode == "dram" else param_device, "nvme_path": path,
                               "pin_memory": True, "buffer_count": 2}}
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
               "zero_optimization": z, "gradient_clipping": 1.0, "aio": {"block_size": 8192, "queue_depth": 4}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        g = torch.Generator().manual_seed(10 + rank)
        for _ in range(3):
            x = torch.randint(0, 97, (2, 12), generator=g)
            eng.backward(eng(x, labels=x))
            eng.step()
        z = eng.optimizer
        if mode == "nvme":
            if opt_device == "nvme":
                assert z.h_master is None and all(v is None for v in z.h_states.values())
                assert z.opt_swapper.bytes_read > 0 and z.opt_swapper.bytes_written > 0
                assert os.path.getsize(z.opt_swapper.files["exp_avg"]) == 4 * z.n_off
            if param_device == "nvme":
                assert z.nvme_param and z.store.lp.numel() == 0
                assert all(u.shard_tensor is None for u in z.units)
                assert os.path.getsize(z.param_swapper.file) >= 4 * z.store.numel // 2
                assert z.param_swapper.bytes_read > 0
            eng.save_checkpoint(d, tag=f"nvme{opt_device}{param_device}")
        res[mode] = z.full_fp32_state_dict(eng._param_names)
    for k in res["dram"]:
        assert torch.equal(res["dram"][k], res["nvme"][k]), k
    # resume from the NVMe-tier checkpoint into a fresh NVMe-tier engine
    torch.manual_seed(1)
    m = LlamaForCausalLM(tiny(**TINY))
    path = os.path.join(d, f"resume{rank}")
    cfg["zero_optimization"]["offload_optimizer"]["nvme_path"] = path
    cfg["zero_optimization"]["offload_param"]["nvme_path"] = path
    eng2, _, _, _ = ds.initialize(model=m, config=cfg)
    eng2.load_checkpoint(d, tag=f"nvme{opt_device}{param_device}")
    got = eng2.optimizer.full_fp32_state_dict(eng2._param_names)
    for k in got:
        assert torch.equal(got[k], res["nvme"][k]), k


def _twin_flow_compact(rank, world, d):
    """Twin-Flow (offload_optimizer.ratio < 1): the device keeps ONE buffer of n + 2m fp32 elements (m = n - n_off)
    under the full-length master / moment views, whose live ranges [n_off, n) are disjoint; the trajectory equals the
    all-device one and a checkpoint round trip restores it exactly."""
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    res = {}
    for mode in ("device", "twin"):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        z = {"stage": 3}
        if mode == "twin":
            z["offload_optimizer"] = {"device": "cpu", "ratio": 0.6}
            z["sub_group_size"] = 20000
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
               "zero_optimization": z, "gradient_clipping": 1.0}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        g = torch.Generator().manual_seed(10 + rank)
        for _ in range(3):
            x = torch.randint(0, 97, (2, 12), generator=g)
            eng.backward(eng(x, labels=x))
            eng.step()
        o = eng.optimizer
        if mode == "twin":
            s, n = o.store, o.store.numel
            mm = n - o.n_off
            assert 0 < o.n_off < n
            base = s.master.untyped_storage().data_ptr()
            assert s.master.untyped_storage().nbytes() == 4 * (n + 2 * mm)
            for i, k in enumerate(("exp_avg", "exp_avg_sq"), 1):
                assert s.states[k].untyped_storage().data_ptr() == base
                assert s.states[k].data_ptr() == base + 4 * i * mm
            eng.save_checkpoint(d, tag=f"twin{world}")
        res[mode] = o.full_fp32_state_dict(eng._param_names)
    for k in res["device"]:  # host Adam vs the fused path: one element of 0.1M lands 1.4e-5 apart
        assert torch.allclose(res["device"][k], res["twin"][k], atol=5e-5), k
    torch.manual_seed(1)
    m = LlamaForCausalLM(tiny(**TINY))
    eng2, _, _, _ = ds.initialize(model=m, config=cfg)
    eng2.load_checkpoint(d, tag=f"twin{world}")
    got = eng2.optimizer.full_fp32_state_dict(eng2._param_names)
    for k in got:
        assert torch.equal(got[k], res["twin"][k]), k
    x = torch.randint(0, 97, (2, 12), generator=torch.Generator().manual_seed(99))
    eng2.backward(eng2(x, labels=x))
    eng2.step()  # the compact layout steps after a load too


@pytest.mark.parametrize("world", [1, 2])
def test_twin_flow_compact_device_part(world, tmp_path):
    run_distributed(_twin_flow_compact, world, str(tmp_path))


@pytest.mark.parametrize("world", [1, 2])
@pytest.mark.parametrize("opt_device,param_device", [("nvme", "cpu"), ("nvme", "nvme"), ("cpu", "nvme")])
def test_zero_infinity_nvme_matches_dram(world, opt_device, param_device, tmp_path):
    run_distributed(_nvme_vs_dram, world, str(tmp_path), opt_device, param_device)


def test_pipelined_swapper_overlap_order(tmp_path):
    """Read-ahead / write-behind bookkeeping: every chunk sees its own data, updates persist, slots never alias."""
    from hcache_deepspeed_amd.ops.aio import aio_handle
    from hcache_deepspeed_amd.runtime.swap_tensor import PipelinedOptimizerSwapper
    sw = PipelinedOptimizerSwapper(aio_handle(4096, 4, False, True, 2), str(tmp_path), ["fp32", "m"], 10_000, 1000)
    base = torch.arange(10_000, dtype=torch.float32)
    sw.write_full("fp32", base)
    sw.write_full("m", None)
    bounds = [(lo, min(lo + 1000, 10_000)) for lo in range(0, 10_000, 1000)] + [(0, 0)][:0]
    bounds = [(0, 700), (700, 1700), (1700, 2000)] + [(lo, lo + 1000) for lo in range(2000, 10_000, 1000)]
    for i, st in sw.pipeline(bounds):
        lo, hi = bounds[i]
        assert torch.equal(st["fp32"], base[lo:hi])
        st["fp32"].add_(1.0)
        st["m"].fill_(float(i))
    assert torch.equal(sw.read_full("fp32"), base + 1)
    m = sw.read_full("m")
    for i, (lo, hi) in enumerate(bounds):
        assert torch.all(m[lo:hi] == i)


def test_refine_plan_closed_loop():
    """The turn-around peak of a planned step corrects the plan: slack keeps the latest spilled layers resident,
    an over-budget peak spills the next layer too."""
    from hcache_deepspeed_amd.offload.activation_cache import refine_plan
    lb = {i: 10 for i in range(8)}
    G = 1 << 30
    assert refine_plan({0, 1, 2, 3, 4}, lb, turn_peak=100, budget=125 + G) == {0, 1, 2}  # 25 B slack: 2 layers
    assert refine_plan({0, 1, 2}, lb, turn_peak=100, budget=105 + G) == {0, 1, 2}        # 5 B: nothing fits
    assert refine_plan({0, 1, 2}, lb, turn_peak=100, budget=95 + G) == {0, 1, 2, 3}      # over budget
    assert refine_plan(set(), lb, turn_peak=100, budget=95 + G) == {0}
    assert refine_plan({0, 1}, lb, turn_peak=0, budget=1000 + G) == set()
    assert refine_plan({0}, lb, turn_peak=100, budget=75 + G) == {0, 1, 2, 3}            # 25 B over: 3 more layers
    assert refine_plan({5, 6}, lb, turn_peak=100, budget=85 + G) == {5, 6, 7}            # runs out of layers


def test_recompute_plans_price_blocks_at_measured_footprint(monkeypatch):
    """Recompute policies: a block that was not checkpointed reports what it kept on the device (allocation growth
    minus its outputs); the plans price every block at least that, so a refinement cannot keep more blocks
    resident than the HBM holds (32k x mb2 ran out of memory when priced at the hook-counted bytes)."""
    import types
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache, refine_plan
    cache = HostActivationCache(torch.device("cpu"), recompute=True)
    cache.n_layers, cache.keep = 8, 2
    cache.device = types.SimpleNamespace(type="cuda")
    alloc = [0]
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda dev=None: alloc[0])
    out = (torch.zeros(4, dtype=torch.bfloat16), torch.zeros(4, dtype=torch.bfloat16))  # 16 B of outputs
    cache.recompute = {0, 1, 2}
    for i, grew in [(1, 1000), (5, 96)]:  # block 1 checkpointed: ignored; block 5 resident: kept 96 - 16 B
        cache._enter(i)
        alloc[0] += grew
        cache._exit(i, out)
    assert cache.resident_block_bytes == 80
    cache._cal_bytes = {i: 50 for i in range(6)}
    assert cache._rc_bytes() == {i: 80 for i in range(6)}
    G = 1 << 30
    # 170 B of slack: 3 blocks at the counted 50 B, but only 2 at the measured 80 B
    assert refine_plan(set(range(6)), cache._cal_bytes, turn_peak=100, budget=270 + G) == {0, 1, 2}
    assert refine_plan(set(range(6)), cache._rc_bytes(), turn_peak=100, budget=270 + G) == {0, 1, 2, 3}
    # calibration: spilled blocks are not measured, the always-resident last blocks are and are never checkpointed
    cache.resident_block_bytes, cache._calibrating, cache.recompute = 0, True, set()
    cache.host_budget, cache.host_in_use, cache._last_layer_bytes = 10, 10, 5
    for i, grew in [(3, 500), (6, 116)]:
        cache._enter(i)
        alloc[0] += grew
        cache._exit(i, out)
    assert cache._cal_recompute == {3} and cache.resident_block_bytes == 100


def test_recompute_policy_wraps_planned_blocks():
    """policy "recompute": the planned blocks run under activation checkpointing (same outputs and gradients,
    no saved activations of their internals), the others are untouched."""
    import torch.nn as nn
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache
    torch.manual_seed(0)
    blocks = nn.ModuleList([nn.Sequential(nn.Linear(16, 16), nn.GELU(), nn.Linear(16, 16)) for _ in range(4)])
    model = nn.Module()
    model.blocks = blocks

    def run(m, x):
        for b in m.blocks:
            x = x + b(x)
        return x.square().sum()

    x = torch.randn(8, 16, requires_grad=True)
    ref = run(model, x)
    ref.backward()
    gref = [p.grad.clone() for p in model.parameters()]
    for p in model.parameters():
        p.grad = None
    cache = HostActivationCache(torch.device("cpu"), recompute=True).attach(model)
    cache.recompute = {0, 2}
    calls = []
    import hcache_deepspeed_amd.runtime.activation_checkpointing.checkpointing as ck
    real = ck.checkpoint

    def spy(fn, *a, **k):
        calls.append(fn)
        return real(fn, *a, **k)

    ck.checkpoint = spy
    try:
        out = run(model, x.detach().requires_grad_(True))
        out.backward()
    finally:
        ck.checkpoint = real
    assert len(calls) == 2
    torch.testing.assert_close(out, ref)
    for p, g in zip(model.parameters(), gref):
        torch.testing.assert_close(p.grad, g)


def test_ckpt_offload_policy_checkpoints_every_block_with_hook_visible_inputs():
    """policy "ckpt_offload": every block is recomputed in backward (same outputs / gradients), and the only tensors
    a block saves are its differentiable INPUTS, passed through save_for_backward -- so an enclosing
    saved_tensors_hooks (the cache's pack hook) sees exactly one input per block."""
    import torch.nn as nn
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache
    torch.manual_seed(0)

    class Block(nn.Module):

        def __init__(self):
            super().__init__()
            self.f = nn.Sequential(nn.Linear(16, 32), nn.GELU(), nn.Dropout(0.3), nn.Linear(32, 16))

        def forward(self, x, scale):
            return x + scale * self.f(x)

    model = nn.Module()
    model.blocks = nn.ModuleList([Block() for _ in range(4)])

    def run(m, x):
        for b in m.blocks:
            x = b(x, 0.5)
        return x.square().sum()

    x = torch.randn(8, 16, requires_grad=True)
    torch.manual_seed(1)
    ref = run(model, x)
    ref.backward()
    gref = [p.grad.clone() for p in model.parameters()]
    gx = x.grad.clone()
    for p in model.parameters():
        p.grad = None
    HostActivationCache(torch.device("cpu"), ckpt_offload=True).attach(model)
    packed = []

    def pack(t):
        packed.append(tuple(t.shape))
        return t

    x2 = x.detach().requires_grad_(True)
    torch.manual_seed(1)  # dropout masks: the recompute replays the forward's RNG state
    with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
        out = run(model, x2)
    out.backward()
    torch.testing.assert_close(out, ref)
    torch.testing.assert_close(x2.grad, gx)
    for p, g in zip(model.parameters(), gref):
        torch.testing.assert_close(p.grad, g)
    # one saved input per block + square()'s input: no internal activation of any block was saved
    assert packed.count((8, 16)) == 5 and len(packed) == 5, packed


def test_pinned_pool_buckets_bound_the_waste():
    """Pinned pool buckets: powers of two up to 64 MiB, 32 MiB granularity above (a 2.68 GB activation must not take
    a 4 GiB buffer: 60 of them overran the host budget at 320k tokens)."""
    from hcache_deepspeed_amd.offload.pinned import PinnedPool
    assert PinnedPool._bucket(1) == 4096
    assert PinnedPool._bucket(5000) == 8192
    assert PinnedPool._bucket(64 << 20) == 64 << 20
    n = 327680 * 4096 * 2
    b = PinnedPool._bucket(n)
    assert b >= n and b - n < (32 << 20) and b % (32 << 20) == 0


def test_auto_policy_splits_recompute_plan_by_pcie_budget():
    """policy "auto": after the first planned (all-recompute) step, the earliest blocks whose D2H fits in
    spill_overlap of the forward move to spilling, the rest stay recomputed."""
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache

    class Ev:
        def __init__(self, ms=0.0):
            self.ms = ms

        def synchronize(self):
            pass

        def elapsed_time(self, other):
            return other.ms - self.ms

    c = HostActivationCache(torch.device("cpu"), hybrid=True, spill_overlap=0.5)
    assert c.policy_recompute and c.hybrid
    G = 1 << 30
    c._cal_bytes = {i: 3 * G for i in range(32)}
    c.recompute = set(range(10))
    c.pcie_gbps = 50.0                    # a 3 GiB block takes ~64 ms
    c._fwd_ev = (Ev(0.0), Ev(900.0))      # 900 ms forward -> 450 ms of copies -> 6 blocks
    c._hybrid_state = 1
    c._hybrid_split()
    assert c.plan == set(range(6)) and c.recompute == set(range(6, 10)) and c._hybrid_state == 2


@pytest.mark.parametrize("stash", [False, True, "host_capped"])
def test_ckpt_offload_attention_stash_exact(stash):
    """policy ckpt_offload with stash_attention: the recompute replays the forward's attention output + LSE instead
    of running attention again -- gradients identical to the plain model; the replay consumes every stashed pair.
    "host_capped": a pinned-host budget that cannot hold the stashes -- no block stashes, attention is recomputed."""
    import torch
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache
    from hcache_deepspeed_amd.ops import attention as A
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(num_hidden_layers=3, vocab_size=128, hidden_size=64, intermediate_size=96,
                              num_attention_heads=4, num_key_value_heads=2, head_dim=16))
    x = torch.randint(0, 128, (2, 16))
    loss = m(x, labels=x)
    loss.backward()
    ref = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    cache = HostActivationCache(torch.device("cpu"), ckpt_offload=True, stash_attention=bool(stash),
                                host_budget_bytes=1 if stash == "host_capped" else None).attach(m)
    stash = stash is True
    calls = {"fwd": 0}
    orig = A._ref_attention

    def counting(*a, **k):
        calls["fwd"] += 1
        return orig(*a, **k)

    A._ref_attention = counting
    try:
        with cache.forward_context():
            loss2 = m(x, labels=x)
        loss2.backward()
    finally:
        A._ref_attention = orig
    assert torch.equal(loss, loss2)
    for n, p in m.named_parameters():
        torch.testing.assert_close(p.grad, ref[n], rtol=0, atol=0, msg=n)
    # 3 blocks: forward once each; the recompute runs attention again only without the stash
    assert calls["fwd"] == (3 if stash else 6), calls
    assert cache.stats()["stashed_blocks"] == (3 if stash else 0)
    assert A.AttnStash.mode is None


def test_stash_keep_and_host_fit_decisions(monkeypatch):
    """ckpt_offload attention stash: blocks stash only while the pinned-host budget holds the stash plus every later
    block's inputs; from the second step the last blocks keep their stash on the device as far as the measured peak
    leaves room (85 % of HBM), and that only grows."""
    import types
    import torch
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache
    GB = 1 << 30
    c = HostActivationCache(torch.device("cpu"), ckpt_offload=True, stash_attention=True, min_layers_resident=1,
                            host_budget_bytes=100 * GB)
    c.n_layers = 10

    class _T:  # stand-in tensor: only sizes matter
        def __init__(self, n):
            self.n = n

        def numel(self):
            return self.n

        def element_size(self):
            return 1

    monkeypatch.setattr(torch, "is_tensor", lambda a: isinstance(a, (_T, torch.Tensor)))
    args = (_T(4 * GB), _T(4 * GB))  # h and residual: 8 GB of inputs, 4 GB hidden -> ~4.08 GB stash
    c.cur_layer, c.host_in_use = 0, 0
    assert c._stash_fits(args)  # 9 blocks x 8 GB + 4.08 <= 100
    c.cur_layer, c.host_in_use = 3, 50 * GB  # 50 + 6 x 8 + 4.08 > 100
    assert not c._stash_fits(args)
    # device keep: steps 1-2 never, then as much as 85 % of HBM minus the peak allows, monotone
    total = 100 * GB
    peak = {"v": 70 * GB}
    c.device = torch.device("cuda")
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: types.SimpleNamespace(total_memory=total))
    import hcache_deepspeed_amd.offload.activation_cache as ac
    monkeypatch.setattr(ac, "log_dist", lambda *a, **k: None)
    c._stash_sb = 4 * GB
    c.last_step_peak = peak["v"]
    c._update_stash_keep()
    assert c.stash_keep_from >= c.n_layers  # not before the second step
    c._update_stash_keep()  # room 85 - 70 = 15 GB -> 3 blocks
    assert c.stash_keep_from == 7
    c.last_step_peak = 84 * GB
    c._update_stash_keep()  # room 1 GB: no change (only grows)
    assert c.stash_keep_from == 7
    c.cur_layer = 8
    assert c._stash_fits(args)  # kept on the device: no host check


def test_step_peak_survives_per_block_resets(monkeypatch):
    """The cache resets the allocator's peak counter at every forward and at every backward block (bwd_headroom).
    The previous step's FULL peak (the max across those resets) is what the stash decision, the calibration and
    peak_gib_all_steps read -- driven through forward_context, whose reset precedes the stash decision."""
    import types
    import torch
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache
    import hcache_deepspeed_amd.offload.activation_cache as ac
    GB = 1 << 30
    alloc = {"cur": 10 * GB, "peak": 10 * GB}

    def set_alloc(v):
        alloc["cur"] = v
        alloc["peak"] = max(alloc["peak"], v)

    def reset(d=None):
        alloc["peak"] = alloc["cur"]

    monkeypatch.setattr(torch.cuda, "max_memory_allocated", lambda d=None: alloc["peak"])
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda d=None: alloc["cur"])
    monkeypatch.setattr(torch.cuda, "reset_peak_memory_stats", reset)
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: types.SimpleNamespace(total_memory=100 * GB))
    monkeypatch.setattr(ac, "log_dist", lambda *a, **k: None)
    c = HostActivationCache(torch.device("cpu"), ckpt_offload=True, stash_attention=True, min_layers_resident=1,
                            gpu_budget_bytes=90 * GB)
    c.device = torch.device("cuda")
    c.n_layers, c._stash_sb = 10, 4 * GB
    for step in range(1):
        with c.forward_context():
            set_alloc(60 * GB)  # forward turn-around: the step's real peak
        # backward: block 9 then 8 -- each new block folds and resets the counter; later blocks peak lower
        c._prefetch_before(9)
        set_alloc(30 * GB)
        c._prefetch_before(8)
        set_alloc(20 * GB)
        c._prefetch_before(7)
        set_alloc(10 * GB)
    with c.forward_context():  # the 2nd forward: decides from step 1's full peak (60), not the last block's (20)
        pass
    assert c.last_step_peak == 60 * GB
    assert c.stats()["peak_gib_all_steps"] == 60.0
    # room 85 - 60 = 25 GB -> 6 blocks of 4 GB keep their stash on the device
    assert c.stash_keep_from == 10 - 6


def test_blit_limit_check_branches(monkeypatch, caplog):
    """A spilling host activation cache warns (strict mode: refuses to start) when DEBUG_CLR_LIMIT_BLIT_WG did not
    reach the HIP runtime (a script that imported torch first); recompute-only, the explicit opt-out and the
    in-effect case pass silently."""
    import logging
    import types
    from hcache_deepspeed_amd.offload.activation_cache import BlitLimitError, check_blit_limit
    monkeypatch.delenv("HDS_ALLOW_UNLIMITED_BLIT", raising=False)
    monkeypatch.delenv("HDS_STRICT_BLIT", raising=False)
    cfg = types.SimpleNamespace(policy="ckpt_offload", allow_unlimited_blit=False)
    check_blit_limit(cfg, "cuda", limit_in_effect=True)
    check_blit_limit(cfg, "cpu", limit_in_effect=False)  # CPU tensors: no blit kernels
    from hcache_deepspeed_amd.utils.logging import logger
    logger.propagate = True
    with caplog.at_level(logging.WARNING):
        check_blit_limit(cfg, "cuda", limit_in_effect=False)  # default: loud warning, run continues
    assert "DEBUG_CLR_LIMIT_BLIT_WG" in caplog.text
    for pol in ("budget", "plan", "auto", "all", "ckpt_offload"):
        with pytest.raises(BlitLimitError, match="DEBUG_CLR_LIMIT_BLIT_WG"):
            check_blit_limit(types.SimpleNamespace(policy=pol, strict_blit_limit=True), "cuda", limit_in_effect=False)
    monkeypatch.setenv("HDS_STRICT_BLIT", "1")
    with pytest.raises(BlitLimitError):
        check_blit_limit(cfg, "cuda", limit_in_effect=False)
    check_blit_limit(types.SimpleNamespace(policy="recompute"), "cuda", limit_in_effect=False)
    check_blit_limit(types.SimpleNamespace(policy="plan", allow_unlimited_blit=True), "cuda", limit_in_effect=False)
    monkeypatch.setenv("HDS_ALLOW_UNLIMITED_BLIT", "1")
    check_blit_limit(cfg, "cuda", limit_in_effect=False)


@pytest.mark.parametrize("order,env,expect", [("torch_first", False, False), ("torch_first", True, True),
                                              ("package_first", False, True)])
def test_blit_limit_detection_by_import_order(order, env, expect):
    """BLIT_LIMIT_EARLY: True iff the variable reached the HIP runtime -- the package imported before torch (it sets
    the variable before the runtime library loads), or the variable exported beforehand."""
    import subprocess
    import sys
    imports = "import torch; import hcache_deepspeed_amd as h" if order == "torch_first" else \
        "import hcache_deepspeed_amd as h; import torch"
    e = {k: v for k, v in os.environ.items() if k != "DEBUG_CLR_LIMIT_BLIT_WG"}
    if env:
        e["DEBUG_CLR_LIMIT_BLIT_WG"] = "16"
    r = subprocess.run([sys.executable, "-c", imports + "; print('EARLY', h.BLIT_LIMIT_EARLY)"], env=e,
                       capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-2000:]
    assert f"EARLY {expect}" in r.stdout, r.stdout


def test_first_plan_keeps_the_copy_window_free():
    """plan_budget: the budget minus the measured backward excess; until a PLANNED step has measured its own excess,
    minus the D2H copy window too (the calibration step it is sized from had nothing in flight at the turn-around).
    step_peaks_gib reports every finished step's peak."""
    import torch
    from hcache_deepspeed_amd.offload.activation_cache import HostActivationCache
    GB = 1 << 30
    c = HostActivationCache(torch.device("cpu"), gpu_budget_bytes=100 * GB, copy_window_bytes=3 * GB)
    assert c.copy_window == 3 * GB
    c.bwd_extra = 2 * GB
    assert c.plan_budget() == 95 * GB  # first plan: budget - excess - window
    c._bwd_extra_planned = 2 * GB
    assert c.plan_budget() == 98 * GB  # a planned step measured its excess: the window margin goes
    c.step_peak_history = [x * GB for x in (10, 50, 60)]
    assert c.stats()["step_peaks_gib"] == [10.0, 50.0, 60.0]
    assert HostActivationCache(torch.device("cpu")).plan_budget() is None


def test_state_offload_shared_allocation_drains_as_one():
    """Tail chunks that are views of ONE allocation (the reload arena, or a whole state split the first time) free
    their HBM only when the last of them drains: the draining queue holds one entry for them, at the last chunk's
    event, with all their bytes; separately allocated chunks keep one entry each."""
    from hcache_deepspeed_amd.runtime.zero.state_offload import OptimizerStateOffload
    issued = [("e0", 10, "arena"), ("e1", 20, "own1"), ("e2", 30, "arena"), ("e3", 5, "own2"), ("e4", 7, "arena")]
    assert OptimizerStateOffload._merge_shared(issued) == [("e1", 20), ("e3", 5), ("e4", 47)]
    assert OptimizerStateOffload._merge_shared([("a", 1, 1), ("b", 2, 2)]) == [("a", 1), ("b", 2)]
