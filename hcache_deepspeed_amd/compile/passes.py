"""DeepCompile schedule passes over the ZeRO-3 unit trace.

Reference parity:
  * compile/passes/zero3_compile.py  -- inserts allgather/release around each parameter use. Here the unit
    trace recorded by the ZeRO-3 optimizer already is that gather/release program (``UnitGraph``);
  * compile/passes/selective_gather.py -- marks the parameters with the highest all-gather time per byte
    persistent while ``total_mem * (1 - margin) - peak_mem`` allows (``selective_gather`` below keeps those
    units gathered from their forward to their backward, removing their backward all-gather);
  * compile/passes/prefetch.py -- reorders all-gathers earlier under a memory limit (``schedule_prefetch``
    below). The reference walks the FX graph backwards and fuses small gathers; fetch units here are already
    flat, coalesced buffers (one all-gather per unit), so the pass only decides WHERE each gather is issued;
  * compile/passes/offload_parameters.py -- parameter shards on pinned host, fetched (H2D + all-gather) at the
    positions the prefetch pass plans; ``plan_param_offload`` keeps the most-fetched shards on the device while
    the HBM budget allows (executed by runtime/zero/optimizer.py ``enable_param_offload``);
  * compile/passes/offload_adam_states.py -- optimizer states to pinned host after the step, back during the
    late backward (``plan_state_reload`` / ``plan_state_offload`` below, executed by
    runtime/zero/state_offload.py). ZeRO-1 needs no schedule here: its flat reduce already runs per unit as each
    unit's gradients complete (the reference's zero1_compile inserts exactly that).

MI355X design: the pass works on measured costs -- per-position compute seconds and live HBM bytes from
``UnitProbe`` and an alpha-beta RCCL all-gather model -- and simulates the single all-gather stream (RCCL runs
the unit gathers of one communicator in issue order). For every gathered unit it picks the LATEST issue
position whose simulated completion still precedes the unit's use: late enough not to hold HBM for longer than
needed, early enough to hide the collective. Units the comm stream cannot hide go as early as memory allows.
On a 288 GB MI355X the memory limit rarely binds for an 8B model, so the pass mostly trades HBM (resident
units) for removed backward gathers, which is what ``selective_gather`` does first.
"""
from collections import defaultdict


class UnitGraph:
    """The unit trace with its measured costs.

    ``fwd``: [(pos, uid, seconds, mem_bytes)] in forward order (pos = index in the forward trace);
    ``bwd``: same for backward (pos = forward index of the unit's backward entry), in backward order;
    ``nbytes``: uid -> gathered bytes; ``gathered``: uids that need an all-gather at all (partitioned units);
    ``peak``: peak allocated bytes of the profiled step; ``total_mem``: device capacity (MIN over ranks)."""

    def __init__(self, fwd, bwd, nbytes, gathered, peak=0, total_mem=0):
        self.fwd = list(fwd)
        self.bwd = list(bwd)
        self.nbytes = dict(nbytes)
        self.gathered = set(gathered)
        self.peak = int(peak)
        self.total_mem = int(total_mem)


class CompiledSchedule:
    """Output of the passes, consumed by the ZeRO-3 optimizer: ``fwd_prefetch[pos]`` / ``bwd_prefetch[pos]``
    list the uids whose all-gather is issued when trace position ``pos`` starts; ``resident`` units are not
    released after their forward (their backward needs no all-gather)."""

    def __init__(self, fwd_prefetch=None, bwd_prefetch=None, resident=(), meta=None):
        self.fwd_prefetch = {int(k): list(v) for k, v in (fwd_prefetch or {}).items()}
        self.bwd_prefetch = {int(k): list(v) for k, v in (bwd_prefetch or {}).items()}
        self.resident = set(resident)
        self.meta = dict(meta or {})

    def to_dict(self):
        return {"fwd_prefetch": self.fwd_prefetch, "bwd_prefetch": self.bwd_prefetch,
                "resident": sorted(self.resident), "meta": self.meta}

    @classmethod
    def from_dict(cls, d):
        return cls(d["fwd_prefetch"], d["bwd_prefetch"], d["resident"], d.get("meta"))


def zero3_compile(graph, resident=()):
    """The gather/release program of one step (reference zero3_compile.py inserts ``allgather_param`` before a
    parameter's first use in a graph and ``release_param`` after its last): a list of
    ``(phase, index, op, uid)`` with op in {"gather", "release"}, ``index`` the position in that phase's
    execution order. A unit used several times in a phase is gathered once before its first use and released
    after its last; ``resident`` units skip the release after their forward and the gather before their backward.
    Returns (program, counts)."""
    prog = []
    counts = {"gathers_fwd": 0, "gathers_bwd": 0, "releases_fwd": 0, "releases_bwd": 0}
    for phase, seq in (("fwd", graph.fwd), ("bwd", graph.bwd)):
        first, last = {}, {}
        for k, (_, uid, _, _) in enumerate(seq):
            if uid in graph.gathered:
                first.setdefault(uid, k)
                last[uid] = k
        for k, (_, uid, _, _) in enumerate(seq):
            if uid not in graph.gathered:
                continue
            skip_gather = phase == "bwd" and uid in resident
            skip_release = phase == "fwd" and uid in resident
            if first[uid] == k and not skip_gather:
                prog.append((phase, k, "gather", uid))
                counts[f"gathers_{phase}"] += 1
            if last[uid] == k and not skip_release:
                prog.append((phase, k, "release", uid))
                counts[f"releases_{phase}"] += 1
    return prog, counts


def plan_param_offload(graph, shard_bytes, budget):
    """Parameter offload (reference compile/passes/offload_parameters.py: every gathered parameter is reloaded from
    the host before its all-gather and offloaded after its last use). The shards live on the host; with HBM to
    spare, keeping a unit's shard on the device removes its host fetches, so the pass keeps the units with the most
    fetches per step (forward + backward gathers of the zero3 program), then the smallest, while their shard bytes
    fit ``budget``. Returns (resident uids, bytes, stats)."""
    prog, _ = zero3_compile(graph)
    fetches = defaultdict(int)
    for _, _, op, uid in prog:
        if op == "gather":
            fetches[uid] += 1
    cands = sorted((uid for uid in shard_bytes if fetches.get(uid)), key=lambda u: (-fetches[u], shard_bytes[u], u))
    res, used = set(), 0
    for uid in cands:
        b = shard_bytes[uid]
        if used + b <= budget:
            res.add(uid)
            used += b
    off = [uid for uid in cands if uid not in res]
    return res, used, {"resident_units": len(res), "resident_bytes": int(used), "offloaded_units": len(off),
                       "offloaded_bytes": int(sum(shard_bytes[u] for u in off)),
                       "host_fetches_per_step": int(sum(fetches[u] for u in off))}


def plan_state_reload(graph, state_bytes, h2d, margin=0.2, mem_limit=None):
    """Placement of the optimizer-state reload (reference offload_adam_states.py: reload tasks in the backward
    graph, early enough to land before the step). Walk the backward from its end and take the LATEST position whose
    remaining backward compute covers the predicted H2D time ``h2d(state_bytes)`` with ``margin`` -- the states
    then hold HBM for as short a time as possible. A position whose live bytes plus the states would exceed
    ``mem_limit`` is skipped towards the end (less hiding, never an OOM). Returns (forward trace position or None,
    stats)."""
    if not graph.bwd or state_bytes <= 0:
        return None, {"h2d_s": 0.0, "covered_s": 0.0}
    t = h2d(state_bytes) * (1.0 + margin)
    tail = 0.0
    k = len(graph.bwd) - 1
    while k > 0 and tail < t:
        tail += graph.bwd[k][2]
        k -= 1
    while mem_limit is not None and k < len(graph.bwd) - 1 and \
            any(m + state_bytes > mem_limit for _, _, _, m in graph.bwd[k:]):
        tail -= graph.bwd[k + 1][2]
        k += 1
    return graph.bwd[k][0], {"h2d_s": t / (1.0 + margin), "covered_s": tail + graph.bwd[k][2],
                             "bwd_index": k, "state_bytes": int(state_bytes)}


def plan_state_offload(graph, state_bytes, d2h):
    """Offload side of the same pass: the D2H is issued right after ``step()`` and overlaps the forward; report how
    much of it the forward's compute covers (the rest delays the release, not compute)."""
    fwd_s = sum(s for _, _, s, _ in graph.fwd)
    t = d2h(state_bytes) if state_bytes > 0 else 0.0
    return {"d2h_s": t, "forward_s": fwd_s, "hidden_frac": 1.0 if t <= 0 else min(1.0, fwd_s / t)}


def selective_gather(graph, predictor, margin=0.1, mem_budget=None):
    """Choose resident units: highest backward all-gather seconds per byte first (ties: shortest distance
    between the unit's forward and backward, i.e. the cheapest HBM-time), while the extra bytes fit into
    ``total_mem * (1 - margin) - peak`` (or ``mem_budget`` when given). Returns (resident set, bytes used)."""
    avail = mem_budget if mem_budget is not None else graph.total_mem * (1.0 - margin) - graph.peak
    if avail <= 0:
        return set(), 0
    fwd_last = {}
    for i, (_, uid, _, _) in enumerate(graph.fwd):
        fwd_last[uid] = i
    bwd_first = {}
    for i, (_, uid, _, _) in enumerate(graph.bwd):
        bwd_first.setdefault(uid, i)
    n = len(graph.fwd)
    cands = []
    for uid in graph.gathered:
        if uid not in bwd_first or uid not in fwd_last:
            continue
        b = graph.nbytes[uid]
        if b <= 0:
            continue
        # positions the unit would stay resident for: the rest of the forward plus the backward up to it
        dist = (n - 1 - fwd_last[uid]) + bwd_first[uid]
        cands.append((-predictor(b) / b, dist, uid))
    cands.sort()
    resident, used = set(), 0
    for _, _, uid in cands:
        b = graph.nbytes[uid]
        if used + b > avail:
            continue
        resident.add(uid)
        used += b
    return resident, used


def schedule_prefetch(seq, predictor, nbytes, mem_limit=None, max_buffered=None):
    """Plan all-gather issue positions for one phase.

    ``seq``: [(pos, uid, seconds, mem_bytes, needs_gather)] in execution order. Returns
    ({pos: [uids]}, stats). A unit is never prefetched before its previous use in the same phase has started
    (it would be released by that use). Without a feasible hiding position the gather goes to the earliest
    position the memory limit and the single comm stream allow."""
    n = len(seq)
    start = [0.0] * (n + 1)
    for k in range(n):
        start[k + 1] = start[k] + seq[k][2]
    extra = [0] * n
    plan = defaultdict(list)
    comm_free = 0.0
    last_issue = 0
    last_use = {}
    hidden = exposed = 0.0
    for k in range(n):
        pos, uid, _, _, needs = seq[k]
        prev = last_use.get(uid)
        last_use[uid] = k
        if not needs or k == 0:
            if needs:
                t = predictor(nbytes[uid])
                comm_free = max(start[k], comm_free) + t
                exposed += t
            continue
        t = predictor(nbytes[uid])
        lo = max(last_issue, (prev + 1) if prev is not None else 0)
        p = None
        for q in range(k - 1, lo - 1, -1):
            if max(start[q], comm_free) + t <= start[k]:
                p = q
                break
        if p is None:
            p = lo
        # memory: the prefetched unit is live from its issue position until its use
        b = nbytes[uid]

        def fits(q):
            for r in range(q, k):
                if mem_limit is not None and seq[r][3] + extra[r] + b > mem_limit:
                    return False
                if max_buffered is not None and extra[r] + b > max_buffered:
                    return False
            return True

        while p < k and not fits(p):
            p += 1
        if p >= k:  # no room: gathered on demand at its use
            fin = max(start[k], comm_free) + t
            exposed += fin - start[k]
            comm_free = fin
            continue
        for r in range(p, k):
            extra[r] += b
        fin = max(start[p], comm_free) + t
        comm_free = fin
        exposed += max(0.0, fin - start[k])
        hidden += t - max(0.0, fin - start[k])
        plan[seq[p][0]].append(uid)
        last_issue = p
    return dict(plan), {"hidden_s": hidden, "exposed_s": exposed, "compute_s": start[n]}


def compile_schedule(graph, predictor, margin=0.1, mem_budget=None, max_buffered=None, selective=True):
    """Run the passes in the reference's order (zero3 -> selective gather -> prefetch) and build the
    ``CompiledSchedule`` the optimizer executes."""
    resident, used = (selective_gather(graph, predictor, margin, mem_budget) if selective else (set(), 0))
    prog, counts = zero3_compile(graph, resident)
    meta = {"zero3": counts}
    meta["selective_gather"] = {"resident_units": len(resident), "resident_bytes": used}
    limit = graph.total_mem * (1.0 - margin) - used if graph.total_mem else None
    # a phase position needs a collective exactly where the gather/release program gathers
    gat = {(ph, k) for ph, k, op, _ in prog if op == "gather"}
    fwd_seq = [(pos, uid, s, m, ("fwd", k) in gat) for k, (pos, uid, s, m) in enumerate(graph.fwd)]
    bwd_seq = [(pos, uid, s, m + used, ("bwd", k) in gat) for k, (pos, uid, s, m) in enumerate(graph.bwd)]
    fwd_plan, fstats = schedule_prefetch(fwd_seq, predictor, graph.nbytes, limit, max_buffered)
    bwd_plan, bstats = schedule_prefetch(bwd_seq, predictor, graph.nbytes, limit, max_buffered)
    meta["prefetch"] = {"fwd": fstats, "bwd": bstats}
    meta["comm_model"] = predictor.to_dict() if hasattr(predictor, "to_dict") else {}
    return CompiledSchedule(fwd_plan, bwd_plan, resident, meta)
