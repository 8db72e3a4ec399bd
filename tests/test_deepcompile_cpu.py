"""DeepCompile schedule passes (hcache_deepspeed_amd/compile/): pass logic on synthetic unit graphs, and the
compiled ZeRO-3 schedule in a world-2 / world-4 gloo run -- identical training trajectory, fewer all-gathers
when units are kept resident, all ranks installing the same schedule.

Reference behaviour: compile/passes/selective_gather.py (persist the highest time-per-byte params within
``total_mem * (1 - margin) - peak``), compile/passes/prefetch.py (move all-gathers earlier under a memory
limit), compile/backend.py (profile then apply passes)."""
import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


def _pred(alpha, bw):
    from hcache_deepspeed_amd.compile import CommPredictor
    return CommPredictor(alpha, bw)


def test_comm_predictor_fit():
    from hcache_deepspeed_amd.compile import CommPredictor
    p = CommPredictor.fit([(1e6, 20e-6 + 1e6 / 1e11), (1e8, 20e-6 + 1e8 / 1e11), (1e9, 20e-6 + 1e9 / 1e11)])
    assert p.alpha == pytest.approx(20e-6, rel=1e-3)
    assert p.beta == pytest.approx(1e11, rel=1e-3)
    assert p(0) == 0.0


def test_prefetch_hides_comm_when_compute_allows():
    from hcache_deepspeed_amd.compile import schedule_prefetch
    # 6 units of 1 ms compute each; each all-gather takes 0.5 ms -> every gather hidden one position ahead
    seq = [(i, i, 1e-3, 0, True) for i in range(6)]
    nbytes = {i: 100 for i in range(6)}
    plan, st = schedule_prefetch(seq, _pred(0.0, 100 / 0.5e-3), nbytes)
    assert plan == {i: [i + 1] for i in range(5)}
    assert st["exposed_s"] == pytest.approx(0.5e-3)  # only the first unit's on-demand gather is exposed
    # gathers of 2.5 ms: the comm stream is the bottleneck -> gathers issued as early as possible
    plan, st = schedule_prefetch(seq, _pred(0.0, 100 / 2.5e-3), nbytes)
    assert plan[0] == [1, 2, 3, 4, 5]
    assert st["exposed_s"] > 0


def test_prefetch_respects_memory_limit_and_reuse():
    from hcache_deepspeed_amd.compile import schedule_prefetch
    seq = [(i, i, 1e-3, 1000, True) for i in range(5)]
    nbytes = {i: 100 for i in range(5)}
    # long gathers want to go early; a limit of one extra unit in flight serialises them one ahead
    plan, _ = schedule_prefetch(seq, _pred(0.0, 100 / 3e-3), nbytes, mem_limit=1100)
    for pos, uids in plan.items():
        assert all(u == pos + 1 for u in uids)
    # a unit used twice is never prefetched before its earlier use has started
    seq = [(0, 7, 1e-3, 0, True), (1, 8, 1e-3, 0, True), (2, 7, 1e-3, 0, True)]
    plan, _ = schedule_prefetch(seq, _pred(0.0, 1e12), {7: 10, 8: 10})
    assert 7 not in plan.get(0, []) and 7 in plan.get(1, [])


def test_selective_gather_budget_and_order():
    from hcache_deepspeed_amd.compile import UnitGraph, selective_gather
    fwd = [(i, i, 1e-3, 0) for i in range(4)]
    bwd = [(i, i, 1e-3, 0) for i in reversed(range(4))]
    g = UnitGraph(fwd, bwd, {0: 100, 1: 100, 2: 100, 3: 100}, {0, 1, 2, 3}, peak=0, total_mem=0)
    res, used = selective_gather(g, _pred(1e-3, 1e9), mem_budget=250)
    # equal time/byte: the units whose backward comes soonest after their forward (the last ones) win
    assert res == {3, 2} and used == 200
    res, _ = selective_gather(g, _pred(1e-3, 1e9), mem_budget=0)
    assert res == set()


def _train(rank, world, compiled, budget, out):
    import os
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
           "zero_optimization": {"stage": 3}, "compile": {"deepcompile": compiled}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    if compiled:
        eng.compile(compile_kwargs={"mem_budget_bytes": budget, "comm_sizes": [4096, 65536]})
    g = torch.Generator().manual_seed(5)
    losses, ags = [], []
    for _ in range(5):
        b = torch.randint(0, 97, (world * 2, 12), generator=g)[rank * 2:(rank + 1) * 2]
        a0 = eng.optimizer.ag_issued
        loss = eng(b, labels=b)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
        ags.append(eng.optimizer.ag_issued - a0)
    sched = eng.optimizer.dc_schedule
    res = {"losses": losses, "ags": ags, "sched": None if sched is None else sched.to_dict()}
    torch.save(res, os.path.join(out, f"r{rank}_{int(compiled)}_{budget}.pt"))


def _run_pair(rank, world, out):
    _train(rank, world, False, None, out)
    _train(rank, world, True, 10**12, out)
    _train(rank, world, True, 0, out)


@pytest.mark.parametrize("world", [2, 4])
def test_deepcompile_zero3_schedule(world, tmp_path):
    run_distributed(_run_pair, world, str(tmp_path))
    load = lambda r, c, b: torch.load(tmp_path / f"r{r}_{c}_{b}.pt", weights_only=True)  # noqa: E731
    for r in range(world):
        base, big, none = load(r, 0, None), load(r, 1, 10**12), load(r, 1, 0)
        # the schedule changes only where gathers happen: the trajectory is bit-identical
        assert big["losses"] == base["losses"] and none["losses"] == base["losses"]
        assert big["sched"] is not None and none["sched"] is not None
        # step 0 records the trace, step 1 is profiled, steps 2.. run the compiled schedule
        assert len(big["sched"]["resident"]) > 0 and none["sched"]["resident"] == []
        assert big["ags"][-1] < base["ags"][-1], (big["ags"], base["ags"])  # no backward re-gathers
        assert none["ags"][-1] == base["ags"][-1]
        assert none["sched"]["fwd_prefetch"] or none["sched"]["bwd_prefetch"]
        # every rank executes the same plan (collective order must match)
        assert big["sched"] == load(0, 1, 10**12)["sched"]


def test_zero3_program_gathers_once_and_skips_resident():
    """The gather/release program: one gather before a unit's first use and one release after its last, per
    phase; resident units keep their forward buffers (no forward release, no backward gather)."""
    from hcache_deepspeed_amd.compile import UnitGraph, zero3_compile
    fwd = [(0, 0, 1e-3, 0), (1, 1, 1e-3, 0), (2, 2, 1e-3, 0), (3, 1, 1e-3, 0)]  # unit 1 used twice
    bwd = [(3, 1, 1e-3, 0), (2, 2, 1e-3, 0), (1, 1, 1e-3, 0), (0, 0, 1e-3, 0)]
    g = UnitGraph(fwd, bwd, {0: 1, 1: 1, 2: 1}, {1, 2}, 0, 0)  # unit 0 persistent (never gathered)
    prog, counts = zero3_compile(g)
    assert counts == {"gathers_fwd": 2, "gathers_bwd": 2, "releases_fwd": 2, "releases_bwd": 2}
    assert ("fwd", 1, "gather", 1) in prog and ("fwd", 3, "release", 1) in prog
    assert ("fwd", 1, "release", 1) not in prog
    _, counts = zero3_compile(g, resident={2})
    assert counts == {"gathers_fwd": 2, "gathers_bwd": 1, "releases_fwd": 1, "releases_bwd": 2}


def test_state_reload_placement():
    """offload_adam_states: the reload is placed where the remaining backward compute covers the H2D time (with
    margin), as late as possible; a memory limit pushes it later."""
    from hcache_deepspeed_amd.compile import UnitGraph, plan_state_reload
    fwd = [(i, i, 1e-3, 0) for i in range(10)]
    bwd = [(i, i, 1e-3, 100) for i in reversed(range(10))]
    g = UnitGraph(fwd, bwd, {i: 1 for i in range(10)}, set(range(10)))
    # H2D 2.5 ms (+20 %): 3 ms of trailing backward compute -> issued 3 positions before the end
    pos, st = plan_state_reload(g, 1000, _pred(0.0, 1000 / 2.5e-3))
    assert pos == 3 and st["covered_s"] >= 3e-3 - 1e-12
    # H2D longer than the whole backward: issued at its start
    pos, _ = plan_state_reload(g, 1000, _pred(0.0, 1000 / 50e-3))
    assert pos == 9
    # live bytes 100 + states 1000 may not exceed 1050 at positions 9..5: the reload moves to position 4
    bwd2 = [(i, i, 1e-3, 100 if i >= 5 else 10) for i in reversed(range(10))]
    g2 = UnitGraph(fwd, bwd2, {i: 1 for i in range(10)}, set(range(10)))
    pos, _ = plan_state_reload(g2, 1000, _pred(0.0, 1000 / 50e-3), mem_limit=1050)
    assert pos == 4


def _state_offload_run(rank, world, stage, out, ratio=1.0, chunk_mb=1024):
    import os
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    res = {}
    for off in (False, True):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        cfg = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 2, "bf16": {"enabled": True},
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": stage},
               "compile": {"offload_opt_states": off}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        if off:
            eng.compile(compile_kwargs={"offload_states_ratio": ratio, "offload_states_chunk_mb": chunk_mb})
        z = eng.optimizer
        g = torch.Generator().manual_seed(5 + rank)
        losses = []
        for step in range(3):
            for _ in range(2):
                x = torch.randint(0, TINY["vocab_size"], (2, 12), generator=g)
                loss = eng(x, labels=x)
                eng.backward(loss)
                eng.step()
                losses.append(float(loss))
            if off:  # between steps the moments' and the fp32 master's tails live on the host only
                so = z.state_offload
                n = z.store.numel
                a = so.a
                assert a == (0 if ratio == 1.0 else min(n, (round((1 - ratio) * n) + 63) // 64 * 64)), (a, n)
                assert z.store.states["exp_avg"].numel() == a and z.store.master.numel() == a
                assert so.state_bytes() == 3 * 4 * (n - a)
                assert all(c is None for cs in so.tail.values() for c in cs)  # every tail chunk off the device
                c = max(64, int(chunk_mb * 2**20) // 4 // 64 * 64)
                assert len(so.bounds) == -(-(n - a) // c) and (so.cuts() or (0, ))[-1] == so.bounds[-1][0]
                assert so.n_offloads == step + 2  # offloaded at compile(), then after every step
        if off:
            assert z.state_offload.n_reloads == 3  # the states start off the device: every step reloads them
        res[off] = losses
        from hcache_deepspeed_amd.utils.tensor_fragment import safe_get_full_fp32_param
        p = next(iter(eng.module.parameters()))
        res[f"w{off}"] = safe_get_full_fp32_param(p).clone()  # reloads on demand
    assert res[False] == res[True]
    assert torch.equal(res["wFalse"], res["wTrue"])


@pytest.mark.parametrize("stage,world,ratio,chunk_mb", [(3, 1, 1.0, 1024), (3, 2, 1.0, 1024), (1, 2, 1.0, 1024),
                                                         (3, 1, 0.3, 1024), (3, 2, 0.55, 1024), (3, 1, 0.55, 0.02),
                                                         (3, 2, 1.0, 0.05)])
def test_offload_adam_states_keeps_trajectory(stage, world, ratio, chunk_mb):
    """Optimizer states and the fp32 master offloaded after every step and reloaded in the next backward: the
    training trajectory is bit-identical to keeping them resident (GAS=2: only the boundary step moves them). With
    ratio < 1 exactly that fraction of every state (its tail) moves and the step runs per piece (byte-granular); small
    ``chunk_mb``: the tail moves as many chunks, each its own piece of the step."""
    run_distributed(_state_offload_run, world, stage, None, ratio, chunk_mb)


def _state_host_step_run(rank, world, ratio):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.utils.tensor_fragment import safe_get_full_fp32_param
    res = {}
    for off in (False, True):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True},
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": 3},
               "compile": {"offload_opt_states": off}, "gradient_clipping": 1.0}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        if off:
            eng.compile(compile_kwargs={"offload_states_ratio": ratio, "offload_states_chunk_mb": 0.05,
                                        "offload_states_host_step": True})
        z = eng.optimizer
        g = torch.Generator().manual_seed(5 + rank)
        losses = []
        for step in range(4):
            x = torch.randint(0, TINY["vocab_size"], (2, 12), generator=g)
            loss = eng(x, labels=x)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
            if off and step == 1:  # a checkpoint-style whole-state read in the middle: the host tails stay current
                safe_get_full_fp32_param(next(iter(eng.module.parameters())))
        if off:
            so = z.state_offload
            assert so.host_step and so.host_steps >= 3 and so.n_reloads <= 1  # only the mid-run whole-state read
            assert z.store.master.numel() == so.a and 0 < so.a < z.store.numel
        res[off] = (losses, torch.cat([safe_get_full_fp32_param(p).flatten() for p in eng.module.parameters()]))
    assert res[True][0] == pytest.approx(res[False][0], rel=1e-3, abs=1e-3)
    # the two Adam kernels round some bf16 parameters one ulp apart after step 1; Adam's sign-like update on the few
    # near-zero gradients this flips then differs by ~lr: a handful of elements, never more than a few steps of lr
    d = (res[True][1] - res[False][1]).abs()
    assert (d > 1e-3).float().mean() < 2e-3 and d.max() < 4e-2, (d.max(), (d > 1e-3).sum())


@pytest.mark.parametrize("world,ratio", [(1, 0.55), (2, 0.4)])
def test_offload_adam_states_host_step(world, ratio):
    """``offload_states_host_step``: the tails never return to the device -- the host Adam updates them in place
    between a gradient D2H and a bf16 parameter H2D per piece, the device kernels update the heads; the trajectory
    follows the resident run (host vs fused Adam: close, not bit-identical), and a whole-state read mid-run (which
    reloads the tails once) leaves the host tails current."""
    run_distributed(_state_host_step_run, world, ratio)


def _state_host_step_fp16_run(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    # dynamic loss scaling starting far too high: the first steps overflow (skipped), later ones step -- every
    # non-skipped step reaches the host tails with a (zero) found_inf flag
    cfg = {"train_micro_batch_size_per_gpu": 2, "fp16": {"enabled": True, "loss_scale": 0, "initial_scale_power": 32,
                    "hysteresis": 1},
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": 3},
           "compile": {"offload_opt_states": True}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    eng.compile(compile_kwargs={"offload_states_ratio": 0.5, "offload_states_chunk_mb": 0.05,
                                "offload_states_host_step": True})
    z = eng.optimizer
    g = torch.Generator().manual_seed(5 + rank)
    applied = 0
    for _ in range(24):
        x = torch.randint(0, TINY["vocab_size"], (2, 12), generator=g)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        applied += int(not z.overflow)
        assert torch.isfinite(loss.float())
    so = z.state_offload
    assert applied >= 1 and so.host_step and so.host_steps >= applied - 1, (applied, so.host_step, getattr(so, "host_steps", 0), so.stats())
    # a set skip flag (symmetric-memory failure, or an overflow folded on the device) leaves the host tails alone
    before = so.host["master"].clone()
    lp = z.store.lp.clone()
    pieces = [(so.a, z.store.numel, z.param_groups[0])]
    so.step_on_host(pieces, 1.0, lp, found_inf=torch.ones(1), lp_cur=z.store.lp)
    assert torch.equal(before, so.host["master"]) and so.host_skips == 1


@pytest.mark.parametrize("world", [1, 2])
def test_offload_adam_states_host_step_fp16_dynamic(world):
    """Host-step tails under fp16 dynamic loss scaling: found_inf is a device flag on every step (it used to send
    the step down the device path, which indexed the host tails' missing device chunks)."""
    run_distributed(_state_host_step_fp16_run, world)


def _resplit_run(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    res = {}
    for mode in ("resident", "resplit"):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True},
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": 3},
               "compile": {"offload_opt_states": mode != "resident"}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        if mode != "resident":
            eng.compile(compile_kwargs={"offload_states_ratio": 1.0, "offload_states_chunk_mb": 0.05,
                                        "offload_states_host_step": True})
        g = torch.Generator().manual_seed(5 + rank)
        losses = []
        for step in range(4):
            x = torch.randint(0, TINY["vocab_size"], (2, 12), generator=g)
            loss = eng(x, labels=x)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
            if mode != "resident" and step == 0:  # what autotune_ratio does after the first (all-host) step
                so = eng.optimizer.state_offload
                assert so.a == 0
                so._resplit(0.4)
                assert 0 < so.a < eng.optimizer.store.numel and eng.optimizer.store.master.numel() == so.a
        res[mode] = losses
    assert res["resplit"] == pytest.approx(res["resident"], rel=1e-3, abs=1e-3)


@pytest.mark.parametrize("world", [1, 2])
def test_state_offload_resplit_after_first_step(world):
    """offload_states_ratio "auto": the first step runs with every state on the host, then the split point moves to
    the ratio the measured peak leaves room for (heads back on the device, tails stay): the trajectory continues."""
    run_distributed(_resplit_run, world)


def test_param_offload_plan():
    """offload_parameters pass: units fetched in both phases are kept on the device first, then the smallest, within
    the budget; units with no fetch are ignored."""
    from hcache_deepspeed_amd.compile import UnitGraph, plan_param_offload, zero3_compile
    fwd = [(i, i, 1e-3, 0) for i in range(4)]
    bwd = [(i, i, 1e-3, 0) for i in (3, 2, 1)]  # unit 0 has no backward (no fetch there)
    g = UnitGraph(fwd, bwd, {i: 100 for i in range(4)}, {0, 1, 2, 3})
    assert len(zero3_compile(g)[0]) == 14
    res, used, st = plan_param_offload(g, {0: 10, 1: 30, 2: 20, 3: 20}, budget=45)
    assert res == {2, 3} and used == 40
    assert st["offloaded_units"] == 2 and st["host_fetches_per_step"] == 3  # unit 1 twice, unit 0 once
    res, used, _ = plan_param_offload(g, {0: 10, 1: 30, 2: 20, 3: 20}, budget=0)
    assert res == set() and used == 0


def _param_offload_run(rank, world, out):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.utils.tensor_fragment import safe_get_full_fp32_param
    res = {}
    # (offload_parameters, mem budget of the passes, offload_opt_states too)
    for mode, (off, budget, states) in {"base": (False, None, False), "all": (True, 0, False),
                                        "some": (True, 80000, False), "everything": (True, 0, True)}.items():
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True},
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": 3},
               "compile": {"deepcompile": off, "offload_parameters": off, "offload_opt_states": states}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        if off:
            eng.compile(compile_kwargs={"mem_budget_bytes": budget, "comm_sizes": [4096, 65536]})
            assert eng.optimizer.offload_param and eng.optimizer.param_offload_gpu_step
        g = torch.Generator().manual_seed(5 + rank)
        losses = []
        for _ in range(5):
            x = torch.randint(0, TINY["vocab_size"], (2, 12), generator=g)
            loss = eng(x, labels=x)
            eng.backward(loss)
            eng.step()
            losses.append(float(loss))
        z = eng.optimizer
        if off:
            meta = z.dc_schedule.meta["offload_parameters"]
            dev = [u.uid for u in z.units if getattr(u, "dev_shard", None) is not None]
            assert sorted(dev) == meta["resident"]
            if budget == 0:
                assert meta["resident_units"] == 0 and meta["offloaded_units"] > 0
            else:
                assert 0 < meta["resident_units"] and meta["offloaded_units"] > 0, meta
        res[mode] = (losses, [safe_get_full_fp32_param(p).clone() for p in eng.module.parameters()])
    for mode in ("all", "some", "everything"):
        assert res[mode][0] == res["base"][0], (mode, res[mode][0], res["base"][0])
        assert all(torch.equal(a, b) for a, b in zip(res[mode][1], res["base"][1])), mode


@pytest.mark.parametrize("world", [1, 2])
def test_offload_parameters_keeps_trajectory(world):
    """compile.offload_parameters on a GPU-optimizer ZeRO-3 engine: shards on the host, fetched by the compiled
    schedule, some kept on the device by the pass under a budget, combined with optimizer-state offload: the training
    trajectory and final weights are bit-identical to the resident run."""
    run_distributed(_param_offload_run, world, None)


def _split_ckpt_run(rank, world, path):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny

    def make(off):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True},
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": 3},
               "compile": {"offload_opt_states": off}}
        eng = ds.initialize(model=m, config=cfg)[0]
        if off:
            eng.compile(compile_kwargs={"offload_states_ratio": 0.5})
        return eng

    g = torch.Generator().manual_seed(11)
    xs = [torch.randint(0, TINY["vocab_size"], (2, 12), generator=g) for _ in range(3)]

    def step(eng, x):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        return float(loss)

    a = make(True)
    for x in xs[:2]:
        step(a, x)
    assert a.optimizer.state_offload.split
    a.save_checkpoint(path, tag="t")  # materializes the split states for the checkpoint
    assert not a.optimizer.state_offload.split
    la = step(a, xs[2])  # re-split by this step's offload
    assert a.optimizer.state_offload.split
    b = make(False)
    b.load_checkpoint(path, tag="t")
    lb = step(b, xs[2])
    assert la == lb, (la, lb)


def test_split_state_offload_checkpoint_roundtrip(tmp_path):
    """Byte-granular state offload: a checkpoint taken while the states are split holds the whole flat states (head
    and tail); an engine without offload resumes from it on the same trajectory."""
    run_distributed(_split_ckpt_run, 1, str(tmp_path))
