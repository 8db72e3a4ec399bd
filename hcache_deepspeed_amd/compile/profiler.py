"""Profiling for the DeepCompile schedule passes: per-position compute time and memory of the ZeRO-3 unit
trace, and an all-gather cost model of the unit communicator.

Reference parity: compile/profilers/graph_profile.py (per-node device time / memory of the traced FX graph)
and compile/profilers/comm_profile.py (``create_predictor``: all-gather time measured over message sizes,
interpolated for the prefetch pass).

MI355X design: there is no FX graph. The "graph" the passes rewrite is the unit execution trace the ZeRO-3
optimizer records on its first step (one node per fetch unit, in forward and backward order). ``UnitProbe``
timestamps each node with a HIP event on the compute stream (host clock on CPU runs) and reads the caching
allocator's live bytes at the same point; the event timestamps are only resolved once, after the profiled
step, so profiling adds no synchronisation to the step itself. The comm model is an alpha-beta fit of
all-gathers on the unit communicator (RCCL over xGMI rings: latency ~tens of us, bandwidth per-link bound),
which is what a ring all-gather costs in the size range of fetch units (tens of MB to a GB).
"""
import time

import torch
import torch.distributed as tdist


class UnitProbe:
    """Collects one forward + backward profile of the unit trace. ``mark(phase, pos)`` is called by the
    optimizer when position ``pos`` of the forward trace starts (forward) or its backward starts; ``end(phase)``
    closes the phase. The first mark of a position wins (a unit whose backward fires more than once)."""

    def __init__(self, device):
        self.cuda = device.type == "cuda"
        self.marks = {"fwd": [], "bwd": []}
        self.ends = {}
        self.seen = {"fwd": set(), "bwd": set()}
        self.peak = 0
        self.active = False
        self.done = False

    def start(self):
        self.marks = {"fwd": [], "bwd": []}
        self.ends = {}
        self.seen = {"fwd": set(), "bwd": set()}
        self.active = True
        if self.cuda:
            torch.cuda.reset_peak_memory_stats()

    def _stamp(self):
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev, torch.cuda.memory_allocated()
        return time.perf_counter(), 0

    def mark(self, phase, pos):
        if not self.active or pos in self.seen[phase]:
            return
        self.seen[phase].add(pos)
        stamp, mem = self._stamp()
        self.marks[phase].append((pos, stamp, mem))

    def end(self, phase):
        if not self.active or phase in self.ends:
            return
        self.ends[phase] = self._stamp()[0]
        if phase == "bwd":
            self.active = False
            self.done = bool(self.marks["fwd"]) and bool(self.marks["bwd"])
            if self.cuda:
                self.peak = torch.cuda.max_memory_allocated()

    def resolve(self):
        """Return {phase: [(pos, seconds, mem_bytes)]} in execution order: the time from a position's mark to
        the next mark (or the phase end)."""
        if self.cuda:
            torch.cuda.synchronize()
        out = {}
        for phase, ms in self.marks.items():
            rows = []
            for i, (pos, st, mem) in enumerate(ms):
                nxt = ms[i + 1][1] if i + 1 < len(ms) else self.ends.get(phase)
                if nxt is None:
                    dt = 0.0
                elif self.cuda:
                    dt = st.elapsed_time(nxt) * 1e-3
                else:
                    dt = nxt - st
                rows.append((pos, max(0.0, dt), mem))
            out[phase] = rows
        return out


class CommPredictor:
    """Alpha-beta model t(bytes) = alpha + bytes / beta of an all-gather on one communicator."""

    def __init__(self, alpha=0.0, beta=float("inf"), samples=()):
        self.alpha = float(alpha)
        self.beta = float(beta)
        self.samples = list(samples)

    def __call__(self, nbytes):
        if nbytes <= 0:
            return 0.0
        return self.alpha + nbytes / self.beta

    def to_dict(self):
        return {"alpha_s": self.alpha, "beta_Bps": self.beta, "samples": self.samples}

    def busbw(self, nbytes, world):
        """nccl-tests bus bandwidth (bytes/s) of an all-gather / reduce-scatter of ``nbytes`` (full buffer):
        (world - 1) / world of the buffer over the predicted time (utils/comms_logging.py factors)."""
        t = self(nbytes)
        return nbytes * (world - 1) / world / t if t > 0 else 0.0

    @staticmethod
    def fit(samples):
        """Least-squares fit of (bytes, seconds) samples; beta is clamped positive."""
        if not samples:
            return CommPredictor()
        if len(samples) == 1:
            b, t = samples[0]
            return CommPredictor(0.0, b / max(t, 1e-9), samples)
        n = len(samples)
        mx = sum(b for b, _ in samples) / n
        my = sum(t for _, t in samples) / n
        sxx = sum((b - mx)**2 for b, _ in samples)
        sxy = sum((b - mx) * (t - my) for b, t in samples)
        slope = sxy / sxx if sxx > 0 else 0.0
        if slope <= 0:  # noisy tiny sizes: bandwidth from the largest sample
            b, t = max(samples)
            return CommPredictor(0.0, b / max(t, 1e-9), samples)
        alpha = max(0.0, my - slope * mx)
        return CommPredictor(alpha, 1.0 / slope, samples)


def profile_allgather(group, device, dtype=torch.bfloat16, sizes_bytes=None, iters=3):
    """Measure all_gather_into_tensor on ``group`` at several per-rank message sizes (all ranks of the group
    must call this together) and fit a ``CommPredictor``. Sizes are total (gathered) bytes."""
    world = tdist.get_world_size(group)
    if world <= 1:
        return CommPredictor()
    if sizes_bytes is None:
        sizes_bytes = ([4 << 20, 32 << 20, 128 << 20, 512 << 20] if device.type == "cuda" else
                       [64 << 10, 512 << 10, 2 << 20])
    esize = torch.empty((), dtype=dtype).element_size()
    samples = []
    for total in sizes_bytes:
        shard = max(1, total // (world * esize))
        inp = torch.empty(shard, dtype=dtype, device=device)
        out = torch.empty(shard * world, dtype=dtype, device=device)
        tdist.all_gather_into_tensor(out, inp, group=group)  # warm the path / communicator
        if device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            tdist.all_gather_into_tensor(out, inp, group=group)
        if device.type == "cuda":
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        # every rank must agree on the model (the schedule is computed identically everywhere): take the max
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX, group=group)
        samples.append((shard * world * esize, float(t.item())))
        del inp, out
    return CommPredictor.fit(samples)


def profile_reduce_scatter(group, device, dtype=torch.bfloat16, sizes_bytes=None, iters=3):
    """Like ``profile_allgather`` for reduce_scatter_tensor (sizes: total input bytes)."""
    world = tdist.get_world_size(group)
    if world <= 1:
        return CommPredictor()
    if sizes_bytes is None:
        sizes_bytes = ([4 << 20, 32 << 20, 128 << 20, 512 << 20] if device.type == "cuda" else
                       [64 << 10, 512 << 10, 2 << 20])
    esize = torch.empty((), dtype=dtype).element_size()
    samples = []
    for total in sizes_bytes:
        shard = max(1, total // (world * esize))
        inp = torch.zeros(shard * world, dtype=dtype, device=device)
        out = torch.empty(shard, dtype=dtype, device=device)
        tdist.reduce_scatter_tensor(out, inp, group=group)
        if device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            tdist.reduce_scatter_tensor(out, inp, group=group)
        if device.type == "cuda":
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX, group=group)
        samples.append((shard * world * esize, float(t.item())))
        del inp, out
    return CommPredictor.fit(samples)


def profile_h2d(device, dtype=torch.bfloat16, sizes_bytes=None, iters=3):
    """ZeRO-Infinity fetches are host->device copies from pinned shards (then an all-gather when sharded):
    measure pinned H2D copies at several sizes and fit a ``CommPredictor`` for them."""
    if device.type != "cuda":
        return CommPredictor()
    sizes_bytes = sizes_bytes or [8 << 20, 64 << 20, 256 << 20]
    esize = torch.empty((), dtype=dtype).element_size()
    samples = []
    for total in sizes_bytes:
        n = max(1, total // esize)
        src = torch.empty(n, dtype=dtype, pin_memory=True)
        dst = torch.empty(n, dtype=dtype, device=device)
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        samples.append((n * esize, (time.perf_counter() - t0) / iters))
        del src, dst
    return CommPredictor.fit(samples)


def combine(a, b):
    """Cost model of a fetch that runs ``a`` then ``b`` (H2D copy of the shard, then its all-gather)."""
    inv = (1.0 / a.beta if a.beta != float("inf") else 0.0) + (1.0 / b.beta if b.beta != float("inf") else 0.0)
    return CommPredictor(a.alpha + b.alpha, 1.0 / inv if inv > 0 else float("inf"), a.samples + b.samples)
