"""Startup self-tuning of the ZeRO-3 unit collectives: which transport carries each (kind, group, size class).

Reference parity: DeepCompile owns its communicator (csrc/compile/deepcompile.cpp:153), issues ``ncclAllGather`` /
``ncclReduceScatter`` on dedicated streams (csrc/compile/z3.cpp:83,235) and can all-gather over symmetric memory
(z3.cpp:91-110) -- each chosen by a config switch. Here nothing is assumed about which is fastest on the node the job
landed on: at data-parallel size > 1 the optimizer measures, for every unit all-gather / reduce-scatter size class of
every group, the three transports this framework has,

* ``rccl``      -- torch.distributed (backend "nccl" = RCCL over xGMI; gloo on CPU dry runs),
* ``native``    -- the private C++ RCCL communicator on a priority stream (comm/native_rccl.py),
* ``symmetric`` -- one-kernel direct-read collectives over IPC-mapped buffers (comm/symmetric.py, one node only),

and routes each size class to the fastest. Every decision is COLLECTIVE: a candidate is usable only if it set up and
produced the reference result on every rank (MIN over the group), and its time is the MAX over the group's ranks, so
all ranks pick the same transport for the same message (a collective that two ranks carried on different transports
would hang). The table -- sizes, per-transport milliseconds, bus bandwidth, choice -- is kept in
``optimizer.comm_selection`` and reported by bench.py in ``extra.comm``.

A transport that fails to set up (no GPU, groups spanning nodes, > 8 ranks for symmetric memory, an RCCL init error)
drops out of the table; rccl is always available.
"""
import time

import torch

from ... import comm as dist
from ...utils.logging import log_dist

TRANSPORTS = ("rccl", "native", "symmetric")


def size_classes(units, lp_es, rs_es, max_classes=3):
    """{(kind, id(group)): (group, [distinct message bytes, largest first])} of the partitioned, non-expert unit
    collectives: all-gathers move the compute-dtype shard, reduce-scatters the padded gradient in the comm dtype."""
    out = {}
    for u in units:
        if u.world <= 1 or getattr(u, "expert_key", None) is not None:
            continue
        for kind, g, nb in (("ag", u.ag_group, u.shard * lp_es), ("rs", u.rs_group, u.padded * rs_es)):
            e = out.setdefault((kind, id(g)), (g, {}))
            e[1][nb] = e[1].get(nb, 0) + 1
    res = {}
    for key, (g, sizes) in out.items():
        # the classes that carry the most bytes per step
        top = sorted(sizes, key=lambda b: -b * sizes[b])[:max_classes]
        res[key] = (g, sorted(top, reverse=True))
    return res


def _flag_device(group, device):
    return device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _agree_min(flag, group, device):
    t = torch.tensor([int(flag)], dtype=torch.int32, device=_flag_device(group, device))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def _agree_max(x, group, device):
    t = torch.tensor([float(x)], dtype=torch.float64, device=_flag_device(group, device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def _shared_device(group, device):
    """True if two ranks of ``group`` drive the same GPU (RCCL refuses such a communicator). Collective."""
    import socket
    me = (socket.gethostname(), torch.cuda.current_device() if device.type == "cuda" else -1)
    ids = [None] * dist.get_world_size(group)
    dist.all_gather_object(ids, me, group=group)
    return len(set(ids)) < len(ids)


class _Timer:
    """Median milliseconds of a collective. On the GPU every timed call runs BESIDE a stream of bf16 GEMMs on a
    second stream (``contend``, default on): in training the unit collectives overlap the compute stream's GEMMs, and
    a transport that takes CUs (the symmetric-memory kernels) or HBM bandwidth pays for it only under that load --
    isolated timing never sees it. ``alone`` keeps the uncontended median of the last call for the table."""

    def __init__(self, cuda, contend=True):
        self.cuda = cuda
        self.contend = bool(contend) and cuda
        self.alone = None
        self._gemm = None

    def _load(self, ms):
        """Queue GEMMs on the side stream covering ~2x ``ms`` of work (the collective then runs under load)."""
        if self._gemm is None:
            a = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
            st = torch.cuda.Stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                torch.mm(a, a)
                e0.record(st)
                for _ in range(4):
                    torch.mm(a, a)
                e1.record(st)
            e1.synchronize()
            self._gemm = (a, st, max(1e-3, e0.elapsed_time(e1) / 4))
        a, st, per = self._gemm
        n = max(2, min(256, int(2 * ms / per) + 2))
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            for _ in range(n):
                torch.mm(a, a)
        return st

    def _one(self, fn, load_ms=None):
        if not self.cuda:
            t0 = time.perf_counter()
            fn()
            return (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        st = self._load(load_ms) if load_ms is not None else None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        if st is not None:
            st.synchronize()
        return e0.elapsed_time(e1)

    def run(self, fn, iters, transport=None):
        """Median milliseconds of ``fn`` (issue + wait), after one untimed call (``transport``: for stub timers)."""
        fn()
        alone = sorted(self._one(fn) for _ in range(iters))
        self.alone = alone[len(alone) // 2]
        if not self.contend:
            return self.alone
        ts = sorted(self._one(fn, load_ms=self.alone) for _ in range(iters))
        return ts[len(ts) // 2]


def _issue(kind, transport, out, inp, group, comm):
    """Issue one collective on ``transport`` and make the current stream wait for it."""
    if transport == "rccl":
        if kind == "ag":
            w = dist.all_gather_into_tensor(out, inp, group=group, async_op=True)
        else:
            w = dist.reduce_scatter_tensor(out, inp, group=group, async_op=True)
        w.wait()
    elif transport == "native":
        (comm.all_gather_into_tensor if kind == "ag" else comm.reduce_scatter_tensor)(out, inp, async_op=True).wait()
    else:  # symmetric: a kernel on the current stream
        if kind == "ag":
            comm.all_gather_into_tensor(out, inp)
        else:
            comm.reduce_scatter_tensor(out, inp)


def _native_factory(kind, group, max_bytes, device):
    if device.type != "cuda":
        raise RuntimeError("needs a GPU")
    if _shared_device(group, device):  # collective, same answer on every rank
        raise RuntimeError("two ranks of the group on one GPU (RCCL refuses a communicator over them)")
    from ...comm.native_rccl import RcclCommunicator
    return RcclCommunicator(group)  # failure-symmetric setup (comm/setup.py)


def _symmetric_factory(kind, group, max_bytes, device):
    if device.type != "cuda":
        raise RuntimeError("needs a GPU")
    from ...comm import symmetric
    if not symmetric.supported(group):  # collective: same-node check
        raise RuntimeError("group is not one node of <= 8 ranks")
    return symmetric.SymmetricMemory(group, max_bytes)  # failure-symmetric setup (comm/setup.py)


# transport -> factory(kind, group, max_bytes, device) -> communicator. A factory may only raise BEFORE its first
# collective if the condition is the same on every rank; after that its collectives must be failure-symmetric.
FACTORIES = {"native": _native_factory, "symmetric": _symmetric_factory}


def _setup(transport, kind, group, max_bytes, device):
    """The communicator object of ``transport`` for ``group`` (None for rccl), or raise."""
    if transport == "rccl":
        return None
    return FACTORIES[transport](kind, group, max_bytes, device)


def select_unit_transports(units, device, lp_dtype, rs_dtype, transports=TRANSPORTS, iters=5, max_symm_bytes=1 << 30,
                           timer=None):
    """Measure every transport on every size class (see module docstring). Returns ``(route, comms, table)``:
    ``route`` {(kind, id(group), bytes): transport}, ``comms`` {(transport, kind, id(group)): communicator object} of
    the transports that won at least one class, ``table`` the JSON-able measurement record. Collective over every
    rank of every unit group, in the same order on every rank."""
    lp_es = torch.empty(0, dtype=lp_dtype).element_size()
    rs_es = torch.empty(0, dtype=rs_dtype).element_size()
    classes = size_classes(units, lp_es, rs_es)
    timer = timer or _Timer(device.type == "cuda")
    route, comms, table = {}, {}, []
    shared = {}  # (transport, id(group)) -> communicator: one native communicator per group serves both kinds
    # insertion order = unit order, identical on every rank (id(group) is not: never sort by it)
    for (kind, gid), (group, sizes) in classes.items():
        world = dist.get_world_size(group)
        dtype = lp_dtype if kind == "ag" else rs_dtype
        es = lp_es if kind == "ag" else rs_es
        avail = {}
        for tr in transports:
            ok, comm, why = True, None, ""
            need = sizes[0]  # a symmetric buffer holds one rank's all-gather shard / one full reduce-scatter input
            if tr == "symmetric" and need > max_symm_bytes:
                ok, why = False, "larger than the symmetric buffer limit"
            if ok:
                try:
                    ck = (tr, gid) if tr == "native" else (tr, kind, gid)
                    comm = shared.get(ck)
                    if comm is None:
                        comm = _setup(tr, kind, group, need, device)
                        shared[ck] = comm
                except Exception as e:  # noqa: BLE001 -- an unavailable transport drops out of the table
                    ok, why = False, f"{type(e).__name__}: {e}"[:160]
            ok = _agree_min(ok, group, device)  # usable only if it set up on EVERY rank
            if ok:
                avail[tr] = comm
            else:
                table.append({"kind": kind, "world": world, "transport": tr, "available": False, "why": why})
        # reference result per size from rccl; a candidate must reproduce it on every rank
        for nb in sizes:
            n = nb // es
            if kind == "ag":
                inp = torch.randn(n, device=device).to(dtype)
                out = torch.empty(n * world, dtype=dtype, device=device)
            else:
                n = (n // world) * world
                inp = torch.randn(n, device=device).to(dtype)
                out = torch.empty(n // world, dtype=dtype, device=device)
            _issue(kind, "rccl", out, inp, group, None)
            ref = out.clone()
            row = {"kind": kind, "world": world, "msg_mib": round(nb / 2**20, 2), "ms": {}, "busbw_GBps": {}}
            for tr, comm in avail.items():
                ok = True
                if tr != "rccl":
                    try:
                        out.zero_()
                        _issue(kind, tr, out, inp, group, comm)
                        if device.type == "cuda":
                            torch.cuda.synchronize()
                        if kind == "ag":  # a gather moves bytes: exact
                            ok = bool(torch.equal(out, ref))
                        else:  # sums in another order / precision (a ring rounds per hop): a broken one is garbage
                            err = (out.float() - ref.float()).norm() / ref.float().norm().clamp_min(1e-30)
                            ok = bool(err < 1e-2)
                    except Exception:  # noqa: BLE001
                        ok = False
                    ok = _agree_min(ok, group, device)
                if not ok:
                    row["ms"][tr] = None
                    continue
                ms = timer.run(lambda tr=tr, comm=comm: _issue(kind, tr, out, inp, group, comm), iters, transport=tr)
                ms = _agree_max(ms, group, device)  # the slowest rank paces a collective
                row["ms"][tr] = round(ms, 4)
                if getattr(timer, "alone", None) is not None and getattr(timer, "contend", False):
                    row.setdefault("ms_alone", {})[tr] = round(_agree_max(timer.alone, group, device), 4)
                # nccl-tests bus-bandwidth factor (W-1)/W of the full message
                row["busbw_GBps"][tr] = round(nb * world * (world - 1) / world / (ms * 1e-3) / 1e9, 1) if ms else None
            timed = {k: v for k, v in row["ms"].items() if v is not None}
            best = min(timed, key=lambda k: (timed[k], k != "rccl"))
            row["choice"] = best
            table.append(row)
            route[(kind, gid, nb)] = best
        for tr, comm in avail.items():
            if tr != "rccl" and any(route.get((kind, gid, nb)) == tr for nb in sizes):
                comms[(tr, kind, gid)] = comm
    # communicators that won nothing are released (symmetric buffers are collective to close)
    used = {id(c) for c in comms.values()}
    for ck, comm in shared.items():
        if comm is not None and id(comm) not in used:
            try:
                if ck[0] == "native":
                    comm.destroy()
                else:
                    comm.close()
            except Exception:  # noqa: BLE001
                pass
    return route, comms, table


def route_for(route, kind, gid, nbytes):
    """The transport of a message: its own size class, else the nearest measured class of the same (kind, group)."""
    tr = route.get((kind, gid, nbytes))
    if tr is not None:
        return tr
    best, dist_best = "rccl", None
    for (k, g, nb), t in route.items():
        if k == kind and g == gid:
            d = abs(nb - nbytes)
            if dist_best is None or d < dist_best:
                best, dist_best = t, d
    return best


def log_table(table):
    for r in table:
        if "choice" in r:
            log_dist(f"zero comm transport: {r['kind']} {r['msg_mib']} MiB x{r['world']}: "
                     + ", ".join(f"{k} {v} ms" for k, v in r["ms"].items()) + f" -> {r['choice']}", ranks=[0])
