"""DeepCompile driver: profile one step of the ZeRO-3 unit trace, run the schedule passes, install the
schedule in the optimizer.

Reference parity: compile/backend.py (``make_backend``: warm-up steps, profiling run of each graph, then the
pass list per graph; ``launch_compile_passes``), compile/init_z3.py (ZeRO-3 setup for compiled graphs) and
csrc/compile/z3.cpp (the executor that runs the scheduled all-gathers / releases / prefetches).

MI355X design: the executor is the ZeRO-3 optimizer itself -- its module hooks issue RCCL all-gathers on the
gather communicator's stream and release buffers on last use; a ``CompiledSchedule`` only changes where
gathers are issued and which units stay resident. Compilation is driven by the training loop:
  step 0            the optimizer records the unit trace (its normal first-step behaviour);
  step ``profile``   ``UnitProbe`` timestamps every trace position (HIP events, no extra syncs);
  after that step    the all-gather cost model is measured on the unit communicator, the passes run, and the
                     schedule (computed on the group's first rank, broadcast so every rank issues collectives
                     in the same order) is installed before the next forward.
With ``dp == 1`` and no parameter offload nothing is gathered and the passes are recorded as no-ops.
"""
import time

import torch
import torch.distributed as tdist

from ..utils.logging import log_dist
from .passes import (CompiledSchedule, UnitGraph, compile_schedule, plan_param_offload, plan_state_offload,
                     plan_state_reload)
from .profiler import CommPredictor, UnitProbe, combine, profile_allgather, profile_h2d


class DeepCompileBackend:

    def __init__(self, engine, profile_step=1, margin=0.1, mem_budget_bytes=None, max_buffered_bytes=None,
                 selective_gather=True, comm_sizes=None):
        self.engine = engine
        self.opt = engine.optimizer
        self.profile_step = int(profile_step)
        self.margin = float(margin)
        self.mem_budget = mem_budget_bytes
        self.max_buffered = max_buffered_bytes
        self.selective = bool(selective_gather)
        self.comm_sizes = comm_sizes
        self.times = {}
        self.schedule = None
        self.graph = None
        self.predictor = None
        self.steps_seen = 0
        self.active = (self.opt is not None and getattr(self.opt, "stage", 0) == 3
                       and getattr(self.opt, "partitioned", False))
        if not self.active:
            self.times["zero1_compile" if getattr(self.opt, "stage", 0) in (1, 2) else "zero3_compile"] = 0.0
            self.meta = {"stage": getattr(self.opt, "stage", 0), "schedule": None,
                         "note": "nothing gathered (ZeRO-1/2, or dp = 1 without parameter offload)"}
            return
        self.probe = UnitProbe(self.opt.device)

    # called by the engine at the end of every optimizer step
    def on_step_end(self):
        if not self.active or self.schedule is not None:
            return
        opt = self.opt
        if self.probe.done:
            self._compile()
            return
        self.steps_seen += 1
        if self.steps_seen >= self.profile_step and not opt._recording and opt._fwd_trace:
            opt.dc_probe = self.probe
            self.probe.start()

    def _group(self):
        for u in self.opt.units:
            if not u.persistent and u.world > 1:
                return u.ag_group
        return self.opt.dp_group

    def _compile(self):
        opt = self.opt
        opt.dc_probe = None
        t0 = time.perf_counter()
        rows = self.probe.resolve()
        trace = opt._fwd_trace
        fwd = [(pos, trace[pos], s, m) for pos, s, m in rows["fwd"] if pos < len(trace)]
        bwd = [(pos, trace[pos], s, m) for pos, s, m in rows["bwd"] if pos < len(trace)]
        esize = torch.empty((), dtype=opt.dtype).element_size()
        nbytes = {u.uid: u.padded * esize for u in opt.units}
        gathered = {u.uid for u in opt.units if not u.persistent and opt._partitioned(u)}
        dev = opt.device
        total = torch.cuda.get_device_properties(dev).total_memory if dev.type == "cuda" else 0
        group = self._group()
        # the plan must be identical on every rank: reduce the profile to its per-position max
        vec = torch.tensor([float(total if total else 1e30), float(self.probe.peak)] + [s for _, _, s, _ in fwd] +
                           [s for _, _, s, _ in bwd] + [float(m) for _, _, _, m in fwd] +
                           [float(m) for _, _, _, m in bwd], dtype=torch.float64, device=dev)
        head = vec[:1].clone()
        tdist.all_reduce(head, op=tdist.ReduceOp.MIN, group=group)
        tdist.all_reduce(vec, op=tdist.ReduceOp.MAX, group=group)
        vals = vec.tolist()
        total = int(head.item()) if total else 0
        peak = int(vals[1])
        nf, nb = len(fwd), len(bwd)
        fs, bs = vals[2:2 + nf], vals[2 + nf:2 + nf + nb]
        fm, bm = vals[2 + nf + nb:2 + 2 * nf + nb], vals[2 + 2 * nf + nb:]
        fwd = [(p, u, fs[i], int(fm[i])) for i, (p, u, _, _) in enumerate(fwd)]
        bwd = [(p, u, bs[i], int(bm[i])) for i, (p, u, _, _) in enumerate(bwd)]
        self.times["profile"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.predictor = profile_allgather(group, dev, opt.dtype, self.comm_sizes)
        if opt.offload_param:
            # ZeRO-Infinity: every fetch is a pinned-host -> HBM copy of the shard first (the all-gather's
            # input is 1/world of the gathered bytes: the copy model is scaled to gathered bytes)
            h2d = profile_h2d(dev, opt.dtype)
            w = max(1, tdist.get_world_size(group) if group is not None else 1)
            h2d = CommPredictor(h2d.alpha, h2d.beta * w, h2d.samples)
            self.predictor = combine(self.predictor, h2d) if self.predictor.beta != float("inf") else h2d
        self.times["comm_profile"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.graph = UnitGraph(fwd, bwd, nbytes, gathered, peak, total)
        budget, pmeta = self.mem_budget, None
        if getattr(opt, "param_offload_gpu_step", False):
            # offload_parameters: the most-fetched shards stay on the device while the headroom allows; a resident
            # world-1 unit needs no fetch at all, so it leaves the gathered set before the other passes run
            head = budget if budget is not None else max(0.0, total * (1.0 - self.margin) - peak) if total else 0.0
            shard = {u.uid: u.shard * esize for u in opt.units if not u.persistent}
            res, used, pstats = plan_param_offload(self.graph, shard, head)
            pmeta = dict(pstats, resident=sorted(res))
            one = {u.uid for u in opt.units if u.world == 1}
            self.graph = UnitGraph(fwd, bwd, nbytes, gathered - (res & one), peak, total)
            budget = max(0.0, head - used)
        sched = compile_schedule(self.graph, self.predictor, self.margin, budget, self.max_buffered,
                                 self.selective)
        if pmeta is not None:
            sched.meta["offload_parameters"] = pmeta
        so = getattr(opt, "state_offload", None)
        if so is not None and dev.type == "cuda":
            # offload_adam_states: the reload goes where the remaining backward covers the measured H2D time
            h2d = profile_h2d(dev, torch.float32)
            nbytes_states = so.state_bytes()
            limit = total * (1.0 - self.margin) if total else None
            pos, rstats = plan_state_reload(self.graph, nbytes_states, h2d, mem_limit=limit)
            sched.meta["offload_adam_states"] = {"reload": rstats,
                                                 "offload": plan_state_offload(self.graph, nbytes_states, h2d)}
            sched.meta["offload_adam_states"]["reload_pos"] = pos
        obj = [sched.to_dict()]
        src = tdist.get_global_rank(group, 0) if group is not None else 0
        tdist.broadcast_object_list(obj, src=src, group=group)
        sched = CompiledSchedule.from_dict(obj[0])
        self.times["passes"] = time.perf_counter() - t0
        if "offload_parameters" in sched.meta:
            opt.set_param_residency(sched.meta["offload_parameters"]["resident"])
        opt.install_schedule(sched)
        if so is not None and "offload_adam_states" in sched.meta:
            so.reload_pos = sched.meta["offload_adam_states"]["reload_pos"]
        self.schedule = sched
        m = sched.meta
        log_dist(f"DeepCompile: {len(trace)} trace positions, resident units "
                 f"{m['selective_gather']['resident_units']} ({m['selective_gather']['resident_bytes'] / 2**30:.2f} "
                 f"GiB), prefetch fwd hidden {m['prefetch']['fwd']['hidden_s'] * 1e3:.2f} ms / exposed "
                 f"{m['prefetch']['fwd']['exposed_s'] * 1e3:.2f} ms, bwd hidden "
                 f"{m['prefetch']['bwd']['hidden_s'] * 1e3:.2f} ms / exposed "
                 f"{m['prefetch']['bwd']['exposed_s'] * 1e3:.2f} ms", ranks=[0])


__all__ = ["DeepCompileBackend", "CommPredictor", "UnitProbe"]
