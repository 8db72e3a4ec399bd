"""ZeRO at the 8-GPU node's rank counts, rehearsed on gloo (VERDICT r1 "Next round" item 1).

* trajectory parity vs torch AdamW at world 4 and 8 for stages 1, 2 and 3 (uneven shard padding at 8:
  the tiny model's units do not divide by 8);
* ZeRO++ hpZ / MiCS / qgZ at world 8 against plain ZeRO-3;
* ZeRO-3 backward memory is bounded: the gathered-parameter + unsharded-gradient bytes the optimizer
  references never exceed a few units, independent of depth (reference stage3.py:372,1305-1308
  ``max_param_reduce_events``), and the coordinator limits (stage3_max_live_parameters,
  stage3_prefetch_bucket_size, stage3_max_reuse_distance) are honoured;
* ``bench.py`` under ``torch.distributed.run --nproc-per-node 4`` (CPU dry run of the multi-rank
  timing / max-over-ranks / JSON path the driver uses on the 8-GPU node).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import _zero_vs_torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stages(rank, world, stages):
    for st in stages:
        _zero_vs_torch(rank, world, st, 1, False)


@pytest.mark.parametrize("world", [4, 8])
def test_zero_stages_parity_large_world(world):
    run_distributed(_stages, world, (1, 2, 3))


def _zeropp8(rank, world):
    from tests.test_zeropp_cpu import _run
    base, _ = _run({})
    hpz, e = _run({"zero_hpz_partition_size": 4})
    assert e.optimizer.hpz == 4
    assert hpz == pytest.approx(base, rel=1e-5, abs=1e-5), (hpz, base)
    mics, e = _run({"mics_shard_size": 4})
    assert e.optimizer.layout_world == 4
    assert mics == pytest.approx(base, rel=1e-4, abs=1e-4), (mics, base)
    qg, e = _run({"zero_quantized_gradients": True})
    assert e.optimizer.qgz
    assert qg == pytest.approx(base, rel=2e-2, abs=2e-2), (qg, base)


def test_zeropp_mics_world8():
    run_distributed(_zeropp8, 8)


DEEP = dict(head_dim=16, hidden_size=64, intermediate_size=128, vocab_size=97, num_attention_heads=4,
            num_key_value_heads=2, num_hidden_layers=10)


def _live_bound(rank, world, inflight, extra):
    os.environ["HDS_ZERO_TRACK_LIVE"] = "1"
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**DEEP))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           "zero_optimization": dict({"stage": 3}, **extra),
           "mi355x": {"zero3_prefetch_depth": 2, "zero3_max_reduce_inflight": inflight}}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    z = eng.optimizer
    layers = [u for u in z.units if not u.persistent]
    assert len(layers) == DEEP["num_hidden_layers"]
    unit_bytes = max(u.padded for u in layers) * z.store.lp.element_size()
    g = torch.Generator().manual_seed(rank)
    peaks = []
    for _ in range(3):  # step 1 records the trace, later steps prefetch from it
        z.live_peak_bytes = 0
        x = torch.randint(0, 97, (2, 12), generator=g)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        peaks.append(z.live_peak_bytes)
        assert not z.pending_rs and not z.pending_works
    # gathered params: current + prefetch_depth units; grads: the current unit's; in flight: ``inflight``
    bound = (1 + 2) * unit_bytes + 1 * unit_bytes + inflight * unit_bytes
    unsharded = 2 * sum(u.padded for u in layers) * z.store.lp.element_size()
    assert max(peaks) <= bound, (peaks, bound, unit_bytes)
    assert max(peaks) < unsharded / 2, (peaks, unsharded)
    return z


def _live_default(rank, world):
    _live_bound(rank, world, 2, {})
    _live_bound(rank, world, 1, {})


@pytest.mark.parametrize("world", [4, 8])
def test_zero3_backward_memory_bounded(world):
    run_distributed(_live_default, world)


def _coordinator_limits(rank, world):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.runtime.zero.flat import NOT_AVAILABLE

    def build(extra):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**DEEP))
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
               "zero_optimization": dict({"stage": 3}, **extra)}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        return eng

    def run(eng, steps=2):
        g = torch.Generator().manual_seed(3)
        out = []
        for _ in range(steps):
            x = torch.randint(0, 97, (2, 12), generator=g)
            loss = eng(x, labels=x)
            out.append(eng.optimizer)
            eng.backward(loss)
            eng.step()
        return [float(v) for v in [loss]]

    base = build({})
    lb = run(base)
    # max_live_parameters of one unit: prefetching is suppressed, so never more than the demanded unit
    # plus the one kept for backward is gathered
    z0 = base.optimizer
    one = max(u.padded for u in z0.units if not u.persistent)
    lim = build({"stage3_max_live_parameters": one})
    seen = []
    orig = lim.optimizer._gather

    def spy(u, wait=True):
        orig(u, wait)
        seen.append(lim.optimizer._live_numel())

    lim.optimizer._gather = spy
    ll = run(lim)
    assert max(seen) <= 3 * one, (max(seen), one)
    assert ll == pytest.approx(lb, rel=1e-5)
    # reuse distance: with a distance covering the last 3 layers, those stay gathered after forward
    per = sum(u.numel for u in z0.units if not u.persistent) // DEEP["num_hidden_layers"]
    reu = build({"stage3_max_reuse_distance": 2 * 2 * per + 1})
    run(reu, 1)
    z = reu.optimizer
    assert len(z._reuse_keep) == 3, z._reuse_keep
    x = torch.randint(0, 97, (2, 12))
    loss = reu(x, labels=x)
    resident = [u.uid for u in z.units if not u.persistent and u.status != NOT_AVAILABLE]
    assert set(resident) >= z._reuse_keep, (resident, z._reuse_keep)
    reu.backward(loss)
    reu.step()
    # prefetch bucket: a bucket smaller than one unit still prefetches exactly one unit ahead
    pb = build({"stage3_prefetch_bucket_size": 1})
    assert run(pb) == pytest.approx(lb, rel=1e-5)


def test_zero3_coordinator_limits_world2():
    run_distributed(_coordinator_limits, 2)


def test_bench_torchrun_cpu_dry_run():
    """bench.py exactly as the driver launches it for N>1 (world 8, as the driver's largest run), on CPU/gloo with
    the tiny preset."""
    W = 8
    env = dict(os.environ, OMP_NUM_THREADS="1", HDS_TUNABLEOP="0", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(W), "--master-addr",
           "127.0.0.1", "--master-port", "29731", os.path.join(ROOT, "bench.py"), "--gpus", str(W), "--steps", "2",
           "--warmup", "1", "--model", "tiny", "--seq", "64", "--micro-batch", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == W and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 2 * W and out["config"]["parallelism"] == f"zero3-dp{W}"
    assert out["value"] > 0 and out["extra"]["valid"] is False
    # communication evidence the driver's N>1 runs carry (exposed wait, per-collective traffic, per-rank HBM)
    comm = out["extra"]["comm"]
    assert comm["ranks"] == W and len(comm["peak_mem_gib_per_rank"]) == W
    assert comm["exposed_comm_ms_per_step_max"] >= 0
    coll = comm["rank0"]["collectives"]
    assert coll["all_gather"]["count"] > 0 and coll["reduce_scatter"]["count"] > 0
    assert coll["all_gather"]["bytes"] > 0 and coll["reduce_scatter"]["world"] == W
    # ZeRO-3 unit events of the instrumented micro-step (reference coordinator events): fetches and waits in both
    # phases, prefetches once the trace is known, with the elements they moved
    ev = comm["unit_events_rank0"]
    for name in ("forward_fetch_wait", "backward_fetch_wait", "forward_prefetch_submit"):
        assert ev[name]["count"] > 0, (name, ev)
    assert ev["forward_prefetch_submit"]["numel"] > 0
    # startup transport measurement: every unit all-gather / reduce-scatter size class timed, one choice each (CPU:
    # only torch.distributed is available; native / symmetric drop out with a reason)
    sel = comm["transport_selection"]
    rows = [r for r in sel if "choice" in r]
    assert {r["kind"] for r in rows} == {"ag", "rs"}
    assert all(r["choice"] == "rccl" and r["ms"]["rccl"] > 0 and r["world"] == W for r in rows)
    assert {r["transport"] for r in sel if r.get("available") is False} == {"native", "symmetric"}
    # the timed steps run uninstrumented; the evidence comes from one extra step and isolated collectives after them
    assert comm["timed_steps_instrumented"] is False and comm["rank0"]["timed_steps_instrumented"] is False
    iso = comm["rank0"]["unit_collectives_isolated"]
    assert iso["all_gather_busbw_GBps"] >= 0 and iso["reduce_scatter"]["samples"]
    # bucket sizes default to "auto" at N > 1: the alpha-beta fit of the data-parallel all-gather is reported
    assert comm["rank0"]["auto_bucket_fit"]["samples"] and comm["rank0"]["xgmi_bucket_mb"] >= 16
    # torchrun forced OMP_NUM_THREADS=1: every rank took its share of the host's CPUs for the host kernels instead
    from hcache_deepspeed_amd.utils.numa import _cgroup_cpu_budget, rank_core_slice
    want = len(rank_core_slice(0, W, budget=_cgroup_cpu_budget()))
    assert comm["host_threads_per_rank"][0] == want and all(t >= 1 for t in comm["host_threads_per_rank"])
    ht = out["extra"]["host_threads"]
    assert ht["source"] == "auto" and ht["local_world"] == W and ht.get("host_kernel_threads", want) == want
    assert out["extra"]["mfu_causal"] <= out["extra"]["mfu_bf16_dense_2.5PF"]


def test_memory_plan_bench_configs():
    """The dp=8 plan of the headline config fits a MI355X; dp=1 matches the measured 244.5 GiB peak."""
    from hcache_deepspeed_amd.models import llama
    from hcache_deepspeed_amd.runtime.zero.mem_estimators import estimate_llama_training
    one = estimate_llama_training(llama.llama3_8b(), 7, 4096, 1)
    assert abs(one["total_gib"] - 244.5) / 244.5 < 0.1, one
    for dp in (2, 4, 8):
        assert estimate_llama_training(llama.llama3_8b(), 7, 4096, dp)["fits"]
    assert estimate_llama_training(llama.llama3_70b(), 1, 4096, 8)["fits"]
    inf = estimate_llama_training(llama.llama3_70b(), 2, 4096, 8, ckpt=True, offload_optimizer=True,
                                  offload_param=True)
    assert inf["fits"] and inf["host_gib"] > 100


def test_comm_stats_drops_completed_works():
    """ZeroCommStats must not retain c10d Work objects (an NCCL Work pins its output tensors, i.e. every gathered
    unit buffer of the timed steps): completed works are accounted and dropped on the next issue, and the number
    retained is bounded even if some never report completion."""
    from hcache_deepspeed_amd.runtime.zero.comm_stats import ZeroCommStats

    class W:

        def __init__(self, done):
            self.done = done

        def is_completed(self):
            return self.done

        def _get_duration(self):
            return 2.0

    cs = ZeroCommStats(torch.device("cpu"))
    for i in range(10):
        cs.issued("all_gather", 1 << 20, 8, W(True))
        assert cs.pending() == 0
    for i in range(300):
        cs.issued("reduce_scatter", 1 << 20, 8, W(False))
    assert cs.pending() <= ZeroCommStats.MAX_PENDING
    s = cs.summary()
    assert s["collectives"]["all_gather"]["count"] == 10 and s["collectives"]["reduce_scatter"]["count"] == 300
    assert s["collectives"]["all_gather"]["busbw_GBps"] > 0 and cs.pending() == 0
