"""Per-step ZeRO collective accounting: how much communication the compute stream actually waited for, and what
bandwidth the all-gathers / reduce-scatters achieved inside the real step.

* **exposed time**: every place the ZeRO optimizer orders the compute stream after a collective
  (``work.wait()`` in ``_gather`` / ``_release`` / ``_retire``) is bracketed by two HIP events on the compute
  stream. Only the wait sits between them, so ``elapsed(before, after)`` is the GPU time compute was stalled on
  communication. (On CPU / gloo, where ``wait()`` blocks the host, the host time of the wait is used.)
* **collective time / busbw**: with ``TORCH_NCCL_ENABLE_TIMING=1`` RCCL records start/end events around every
  collective kernel; ``Work._get_duration()`` reads them after the step. busbw uses the nccl-tests factors of
  utils/comms_logging.py (all-gather and reduce-scatter: ``(n-1)/n`` of the full buffer per unit time).

Enabled by ``mi355x.comm_stats`` (bench.py turns it on at N > 1). Reference counterpart: the comms logger's
per-op latency/algbw/busbw (utils/comms_logging.py:33-178), which synchronizes around every op; this one does not
synchronize inside the step.
"""
import time

import torch


def _completed(work):
    """Non-blocking completion check of a c10d / event-backed work object (unknown kinds count as complete)."""
    f = getattr(work, "is_completed", None)
    if f is not None:
        try:
            return bool(f())
        except Exception:
            return True
    ev = getattr(work, "ev", None)
    if ev is not None and hasattr(ev, "query"):
        return bool(ev.query())
    return True


class ZeroCommStats:
    """Work objects are accounted and DROPPED as soon as they complete: a c10d NCCL Work keeps its output tensors
    alive (``outputs_``), so holding every step's works until ``summary()`` would pin each freshly gathered unit
    buffer -- 14 GB per step for Llama-3-8B -- for the whole timed region."""

    MAX_PENDING = 64  # hard bound on retained works; older ones are accounted without timing

    def __init__(self, device):
        self.device = device
        self.cuda = device.type == "cuda"
        self.reset()

    def reset(self):
        self._waits = []  # (ev_before, ev_after) or host seconds
        self._works = []  # (kind, total_bytes, world, work) not yet complete
        self._kinds = {}
        self.host_wait_s = 0.0

    def _account(self, kind, nbytes, world, work, timed=True):
        d = self._kinds.setdefault(kind, {"count": 0, "bytes": 0, "timed_ms": 0.0, "timed_bytes_bus": 0.0,
                                          "world": world})
        d["count"] += 1
        d["bytes"] += nbytes
        ms = None
        if timed:
            try:
                ms = float(work._get_duration())
            except Exception:  # timing not enabled (TORCH_NCCL_ENABLE_TIMING) or not supported by the backend
                ms = None
        if ms is not None and ms > 0:
            d["timed_ms"] += ms
            d["timed_bytes_bus"] += nbytes * (world - 1) / world

    def _drain(self, all_done=False):
        keep = []
        for item in self._works:
            if all_done or _completed(item[3]):
                self._account(*item)
            else:
                keep.append(item)
        while len(keep) > self.MAX_PENDING:
            self._account(*keep.pop(0), timed=False)
        self._works = keep

    def issued(self, kind, total_bytes, world, work):
        if world > 1 and work is not None:
            self._works.append((kind, int(total_bytes), int(world), work))
            self._drain()

    def wait(self, work):
        if not self.cuda:
            t0 = time.perf_counter()
            work.wait()
            self.host_wait_s += time.perf_counter() - t0
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        work.wait()
        e1.record()
        self._waits.append((e0, e1))

    def pending(self):
        return len(self._works)

    def summary(self):
        """Call after the step's work has completed (e.g. after ``torch.cuda.synchronize()``)."""
        self._drain(all_done=True)
        if self.cuda:
            exposed_ms = sum(a.elapsed_time(b) for a, b in self._waits)
        else:
            exposed_ms = self.host_wait_s * 1e3
        out = {"exposed_ms": round(exposed_ms, 3), "waits": len(self._waits) if self.cuda else None}
        kinds = {}
        for kind, d0 in self._kinds.items():
            d = dict(d0)
            ms, bus = d.pop("timed_ms"), d.pop("timed_bytes_bus")
            d["collective_ms"] = round(ms, 3) if bus else None
            d["busbw_GBps"] = round(bus / (d["collective_ms"] * 1e-3) / 1e9, 1) if d["collective_ms"] else None
            d["mean_msg_MiB"] = round(d["bytes"] / max(1, d["count"]) / 2**20, 2)
            kinds[kind] = d
        out["collectives"] = kinds
        return out


class UnitEventProfiler:
    """Host-side counts and durations of ZeRO-3 unit events (fetch, prefetch, wait, release) with the elements each
    moved; the API of the reference's partitioned-parameter profiler (runtime/zero/partitioned_param_profiler.py:10),
    kept next to the collective accounting above. ``timers`` (utils/timer.SynchronizedWallClockTimer) optionally
    receives the same start/stop calls so the events appear in the engine's timer log."""

    class _Event:
        __slots__ = ("name", "count", "num_elem", "seconds", "_t0")

        def __init__(self, name):
            self.name, self.count, self.num_elem, self.seconds, self._t0 = name, 0, 0, 0.0, None

    def __init__(self, timers=None):
        self.timers = timers
        self.event_counters = {}

    def reset_events(self):
        self.event_counters = {k: self._Event(k) for k in self.event_counters}

    def start_event(self, name):
        ev = self.event_counters.get(name)
        if ev is None:
            ev = self.event_counters[name] = self._Event(name)
        ev._t0 = time.perf_counter()
        if self.timers is not None:
            self.timers(name).start()

    def cancel_event(self, name):
        """Drop a started event that moved nothing (the reference records prefetch events only when it issues)."""
        ev = self.event_counters.get(name)
        if ev is not None:
            ev._t0 = None

    def stop_event(self, name, num_elem):
        ev = self.event_counters.get(name)
        if ev is None or ev._t0 is None:
            raise KeyError(f"stop_event({name!r}) without a matching start_event")
        ev.seconds += time.perf_counter() - ev._t0
        ev._t0 = None
        ev.count += 1
        ev.num_elem += int(num_elem)
        if self.timers is not None:
            self.timers(name).stop()

    def summary(self):
        return {k: {"count": e.count, "numel": e.num_elem, "ms": round(e.seconds * 1e3, 3)}
                for k, e in self.event_counters.items()}

    def log_events(self):
        from ...utils.logging import log_dist
        parts = [f"{k}: {d['count']}x {d['numel']} elem {d['ms']} ms" for k, d in self.summary().items()]
        log_dist("zero-3 unit events | " + " | ".join(parts), ranks=[0])
        if self.timers is not None and self.event_counters:
            self.timers.log(names=list(self.event_counters))
