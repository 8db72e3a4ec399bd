"""Asynchronous optimizer-state offload between steps: the executor of DeepCompile's ``offload_adam_states`` pass.

Reference parity: compile/passes/offload_adam_states.py (offload tasks after the optimizer step on a copy stream,
per-key events, reload tasks placed in the backward graph so the states are back by the step) and
csrc/compile/z3.cpp:268-341 (dedicated offload / reload streams); the byte fraction of ZeRO-Offload's Twin-Flow
``ratio`` (runtime/zero/offload_config.py:93, stage3.py:120-136).

MI355X design: every state is a flat buffer of this rank's shard (runtime/zero/flat.py ``ShardStore``). With
``ratio`` r the executor SPLITS each moved state (the Adam moments and the fp32 master) at element a = (1 - r) * n
into two separately allocated pieces:

* the head [0, a) stays on the device for good (``store.states[k]`` / ``store.master`` ARE the heads while split);
* the tail [a, n) lives in pinned host memory between ``step()`` and the late backward of the next step: one D2H per
  state on a high-priority copy stream right after the step (overlapping the next forward), its device buffer
  released the moment the DMA drains; the reload is issued at the backward trace position the pass picks
  (``compile/passes.plan_state_reload``) or as soon as the HBM the backward has freed holds it.

``step()`` runs the fused optimizer kernel per contiguous piece (``cuts()``: the step splits its segments at a), so
the states are never concatenated: exactly r of the state bytes cross PCIe each way per step -- byte-granular, not
whole 32 GB states (round 4). r = 1 moves everything (a = 0). Readers that need whole flat states (checkpoints,
``safe_get_full_fp32_param``) call ``wait()``, which materializes them (head ++ tail, one device concatenation) and
leaves them whole until the next step's ``offload()`` splits them again.

The tail is moved in CHUNKS of ``chunk_mb`` (default 1 GiB; ``cuts()`` includes every chunk boundary, so the step
still runs per contiguous piece):

* each chunk's HBM returns to the allocator as soon as ITS D2H drains (the allocator polls the copy events at every
  allocation), so the next forward's activations grow into the memory the offload frees, chunk by chunk, instead of
  waiting for a whole 10-30 GB state; at every forward unit ``on_forward_position()`` waits for just enough of the
  oldest chunks to drain to hold that unit's activations (the growth measured on the previous step) -- an allocation
  that found nothing free would otherwise make the allocator synchronize EVERY outstanding copy at once;
* the backward reloads the tails as soon as the HBM it has freed holds them -- in ONE allocation (sliced per chunk):
  chunk-by-chunk reloads into the holes of a half-freed activation pool fragmented it for the next forward.

``host_step`` (``offload_states_host_step``): the tails never come back. They stay in pinned host memory and ``step()``
updates them THERE with the host Adam -- per piece, the gradient goes D2H, the host kernel updates master and moments
in place and writes the bf16 parameters into pinned staging, which goes H2D -- while the device kernels update the
heads. Per step r x 2 bytes per element cross PCIe each way with bf16 gradients (r x 4 down with fp32 ones) instead of
r x 12 (the Twin-Flow split of ZeRO-Offload, applied to the pass's byte-granular tails); nothing is reloaded before
``step()`` and nothing is offloaded after it.

Offload and reload run on SEPARATE copy streams: a reload issued while the post-step offload of other chunks is still
draining does not queue behind it -- it waits only for its own chunk's offload.
"""
import collections
import os

import torch


class OptimizerStateOffload:

    def __init__(self, zopt, include_master=True, ratio=1.0, chunk_mb=1024, host_step=False):
        self.z = zopt
        self.include_master = bool(include_master)
        self.host_step = bool(host_step) and self.include_master and zopt.kind == "adam"
        self._h_grad = self._h_lp = None  # host-step staging (pinned, double-buffered)
        self._h_grad_full = self._h_lp_full = None  # async host step: pinned staging of the whole tail
        self._async = None  # the in-flight async host step (see step_on_host)
        self._unit_pieces = {}
        self._thread = None
        # "auto" (reference compile/passes/offload_adam_states.py:253 decides from profiled memory): the first step
        # runs with everything on the host, then ``autotune_ratio`` keeps on the device what its measured peak leaves
        # room for
        self.auto_ratio = str(ratio) == "auto"
        self.auto_info = None
        self.ratio = 1.0 if self.auto_ratio else min(1.0, max(0.0, float(ratio)))
        self.chunk_bytes = max(256, int(float(chunk_mb) * 2**20))
        dev = zopt.device
        self.cuda = dev.type == "cuda"
        self.stream = torch.cuda.Stream(dev, priority=-1) if self.cuda else None  # offload (D2H)
        self.reload_stream = torch.cuda.Stream(dev, priority=-1) if self.cuda else None  # reload (H2D)
        self.host = {}  # key -> pinned tail [n - a]
        self.tail = {}  # key -> [device chunk or None (off the device)] per tail chunk
        self.events = {}  # (key, chunk) -> last D2H / H2D event of that chunk
        self.split = False  # heads + tail chunks (not whole flat states)
        self.offloaded = False  # tail chunks (some) off the device, not all reloaded yet
        self.reloading = False
        self.reload_pos = None  # backward trace position that triggers the reload (None: backward start)
        self.a = None  # split element
        self.bounds = []  # [(lo, hi)] element ranges of the tail chunks, lo of the first = a
        self.bytes = 0
        self.n_offloads = 0
        self.n_reloads = 0
        self._draining = collections.deque()  # (event, bytes) of chunks whose D2H may still run, oldest first
        self._fwd_growth = 0  # largest per-unit growth of allocated HBM in the last forward (bytes)
        self._fwd_last = None
        self.fwd_waits = 0  # chunk drains the forward waited for (last step)
        self.fwd_wait_s = 0.0

    # -----------------------------------------------------------------------------------------------------
    def _keys(self):
        """State keys this executor moves: the device-resident moments (host-resident ones -- ZeRO-Offload -- are left
        alone) and the fp32 master unless it IS the compute-dtype shard (fp32 training)."""
        s = self.z.store
        keys = [k for k, v in s.states.items() if v is not None and v.device.type == self.z.device.type]
        m = s.master
        if (self.include_master and m is not None and m.device.type == self.z.device.type
                and not (m.numel() and s.lp.numel() and m.data_ptr() == s.lp.data_ptr())):
            keys.append("master")
        return keys

    def _get(self, k):
        s = self.z.store
        return s.master if k == "master" else s.states[k]

    def _set(self, k, t):
        s = self.z.store
        if k == "master":
            s.master = t
        else:
            s.states[k] = t

    def _split_at(self, n, es=4):
        if self.a is None:
            a = int(round((1.0 - self.ratio) * n))
            self.a = min(n, (a + 63) // 64 * 64) if a > 0 else 0  # 256-B aligned pieces for the vector kernels
            c = max(64, self.chunk_bytes // es // 64 * 64)
            self.bounds = [(lo, min(n, lo + c)) for lo in range(self.a, n, c)]
        return self.a

    def cuts(self):
        """Element offsets at which ``step()`` must split its ranges: the head/tail boundary and every chunk
        boundary while split."""
        if not self.split:
            return ()
        return tuple(lo for lo, _ in self.bounds if lo > 0)

    def _chunk_of(self, lo):
        c = self.bounds[0][1] - self.bounds[0][0]
        return (lo - self.a) // c

    def view(self, k, lo, hi):
        """[lo, hi) of state ``k`` (``k`` = "master" or a moment key) inside ONE piece (never across a cut)."""
        if not self.split or k not in self.host:  # not split, or a state this executor does not move
            return self._get(k)[lo:hi]
        if hi <= self.a:
            return self._get(k)[lo:hi]
        assert lo >= self.a, "a range across the head/tail cut"
        i = self._chunk_of(lo)
        c0, c1 = self.bounds[i]
        assert hi <= c1, "a range across a tail chunk boundary"
        return self.tail[k][i][lo - c0:hi - c0]

    def moves(self, k):
        return k in self.host or (not self.split and k in self._keys())

    def state_bytes(self):
        """Bytes one offload moves each way."""
        if self.host:
            return sum(h.numel() * h.element_size() for h in self.host.values())
        n = self.z.store.numel
        return sum((n - self._split_at(n, self._get(k).element_size())) * self._get(k).element_size()
                   for k in self._keys())

    # -----------------------------------------------------------------------------------------------------
    def offload(self):
        """After ``step()``: D2H every tail chunk on the copy stream; each chunk's HBM returns to the allocator when
        its own DMA drains. Whole (materialized) states are split first: the head is a new allocation."""
        if self.offloaded:
            return
        self.bytes = 0
        cur = torch.cuda.current_stream() if self.cuda else None
        # retire drained entries (engines without per-unit forward hooks never call on_forward_position)
        self._draining = collections.deque((e, nb) for e, nb in self._draining if not e.query())
        if self.cuda:
            self.stream.wait_stream(cur)
        keys = self._keys() if not self.split else list(self.host)
        issued = []  # (event, bytes, storage) in D2H order: chunks that are views of ONE allocation (a reload arena,
        # or a whole state split for the first time) free their HBM only when the LAST of them drains
        for k in keys:
            if self.split:
                chunks, head = self.tail.get(k), None
                if chunks is None:
                    continue
            else:  # whole flat state -> head (stays) + tail chunks (go)
                full = self._get(k)
                n = full.numel()
                if n == 0:
                    continue
                a = self._split_at(n, full.element_size())
                head = full[:a].clone() if a else full.new_empty(0)
                chunks = [full[lo:hi] for lo, hi in self.bounds]  # views: the whole buffer goes with the last one
            a = self.a
            h = self.host.get(k)
            if h is None or h.numel() != self.z.store.numel - a:
                h = self.host[k] = torch.empty(self.z.store.numel - a, dtype=chunks[0].dtype if chunks else torch.float32,
                                               pin_memory=self.cuda)
            for i, t in enumerate(chunks):
                if t is None:
                    continue
                lo, hi = self.bounds[i]
                nb = t.numel() * t.element_size()
                if self.cuda:
                    with torch.cuda.stream(self.stream):
                        h[lo - a:hi - a].copy_(t, non_blocking=True)
                        t.record_stream(self.stream)  # the block recycles only after ITS DMA drained
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    self.events[(k, i)] = ev
                    issued.append((ev, nb, t.untyped_storage().data_ptr()))
                else:
                    h[lo - a:hi - a].copy_(t)
                self.bytes += nb
            self.tail[k] = [None] * len(self.bounds)
            del chunks
            if head is not None:
                self._set(k, head)
        self._draining.extend(self._merge_shared(issued))
        self.split = True
        self.offloaded = True
        self.reloading = False
        self.n_offloads += 1
        self._fwd_last = None
        self.fwd_waits, self.fwd_wait_s = 0, 0.0

    @staticmethod
    def _merge_shared(issued):
        """[(event, bytes, storage)] in issue order -> [(event, bytes)] with every group of chunks that share one
        allocation merged into ONE entry at its last chunk's position: its bytes become usable only when that last
        D2H drains (``record_stream`` on each view pins the whole block until then)."""
        last, total = {}, collections.Counter()
        for j, (_, nb, st) in enumerate(issued):
            last[st] = j
            total[st] += nb
        return [(ev, total[st]) for j, (ev, _, st) in enumerate(issued) if last[st] == j]

    def start_profile(self):
        """Reset the allocator peak once the states have left the device (the first step's peak is then the
        activations' and the step's, which ``autotune_ratio`` sizes the resident heads against)."""
        if self.cuda and self.auto_ratio:
            torch.cuda.synchronize(self.z.device)
            torch.cuda.reset_peak_memory_stats(self.z.device)

    def autotune_ratio(self, margin_gib=6.0):
        """After the first (all-offloaded) step: the fraction of the states that must stay off the device so the
        resident heads plus the measured peak fit ``mem_fraction`` of HBM with ``margin_gib`` to spare, rounded up
        to 5 %. The heads move back to the device once; the tails keep stepping where they were."""
        if not self.auto_ratio or self.auto_info is not None or not self.cuda:
            return None
        self.join()
        dev = self.z.device
        torch.cuda.synchronize(dev)
        peak = torch.cuda.max_memory_allocated(dev)
        limit = int(self.mem_fraction * torch.cuda.get_device_properties(dev).total_memory)
        state_bytes = sum(h.numel() * h.element_size() for h in self.host.values())
        free = max(0, limit - peak - int(margin_gib * 2**30))
        import math
        r = 1.0 - (free / state_bytes if state_bytes else 0.0)
        r = min(1.0, max(0.0, math.ceil(r * 20 - 1e-9) / 20))
        self.auto_info = {"peak_gib_step1": round(peak / 2**30, 1), "limit_gib": round(limit / 2**30, 1),
                          "state_gib": round(state_bytes / 2**30, 1), "ratio": r}
        if r < 1.0:
            self._resplit(r)
        return r

    def _resplit(self, ratio):
        """Move the split point from a = 0 (everything on the host) to (1 - ratio) * n: the heads [0, a') come back to
        the device (one H2D each), the host tails become views past a' of the same pinned buffers."""
        assert self.split and self.a == 0 and self.offloaded
        n = self.z.store.numel
        a = int(round((1.0 - ratio) * n))
        a = min(n, (a + 63) // 64 * 64)
        for k in list(self.host):
            h = self.host[k]
            head = torch.empty(a, dtype=h.dtype, device=self.z.device)
            head.copy_(h[:a])
            self._set(k, head)
            self.host[k] = h[a:]
        es = 4
        c = max(64, self.chunk_bytes // es // 64 * 64)
        self.a, self.ratio = a, ratio
        self.bounds = [(lo, min(n, lo + c)) for lo in range(a, n, c)]
        self.tail = {k: [None] * len(self.bounds) for k in self.host}
        self.events = {}
        self._h_grad_full = self._h_lp_full = None
        self._h_grad = self._h_lp = None
        if self.cuda:
            torch.cuda.synchronize(self.z.device)

    def on_forward_position(self):
        """Before a forward unit runs: retire the drained chunks and, if the HBM the allocator can hand out does not
        hold this unit's activation growth (measured on the previous forward), wait for the oldest draining chunks --
        just enough of them -- instead of letting a failed allocation synchronize every outstanding copy."""
        if not self.cuda:
            return
        dq = self._draining
        while dq and dq[0][0].query():
            dq.popleft()
        alloc = torch.cuda.memory_allocated(self.z.device)
        if self._fwd_last is not None:
            self._fwd_growth = max(self._fwd_growth, alloc - self._fwd_last)
        self._fwd_last = alloc
        if not dq:
            return
        need = 2 * self._fwd_growth + (1 << 30) if self._fwd_growth else 4 << 30
        free, _ = torch.cuda.mem_get_info(self.z.device)
        draining = sum(nb for _, nb in dq)
        usable = free + max(0, torch.cuda.memory_reserved(self.z.device) - alloc - draining)
        if usable >= need:
            return
        import time
        t0 = time.perf_counter()
        while dq and usable < need:
            ev, nb = dq.popleft()
            ev.synchronize()
            usable += nb
            self.fwd_waits += 1
        self.fwd_wait_s += time.perf_counter() - t0

    def _pending(self):
        """(key, chunk) of the tail chunks still off the device, largest states first."""
        if not self.offloaded:
            return []
        return [(k, i) for k in self.host for i in range(len(self.bounds)) if self.tail[k][i] is None]

    def _chunk_bytes(self, k, i):
        lo, hi = self.bounds[i]
        return (hi - lo) * self.host[k].element_size()

    def reload(self, keys=None, chunks=None):
        """Issue the H2D of the offloaded tail chunks (all, those of ``keys``, or the (key, chunk) pairs ``chunks``;
        non-blocking); ``wait_tails()`` orders the compute stream after them."""
        if not self.offloaded or self.reloading:
            return
        cur = torch.cuda.current_stream() if self.cuda else None
        ready = None
        todo = chunks if chunks is not None else [(k, i) for k, i in self._pending() if keys is None or k in keys]
        todo = [(k, i) for k, i in todo if self.tail[k][i] is None]
        # ONE allocation for the chunks of this call, sliced per chunk: reloading chunk by chunk into the holes the
        # backward frees scattered 1 GiB blocks among the activations, and the next forward found 40 GiB free but no
        # 2 GiB in one piece (this allocator has no expandable segments on ROCm)
        dts = {self.host[k].dtype for k, _ in todo}
        arena = None
        if self.cuda and len(dts) == 1 and len(todo) > 1:
            arena = torch.empty(sum(self.bounds[i][1] - self.bounds[i][0] for _, i in todo), dtype=dts.pop(),
                                device=self.z.device)
        off = 0
        for k, i in todo:
            lo, hi = self.bounds[i]
            h = self.host[k][lo - self.a:hi - self.a]
            if arena is not None:
                buf = arena[off:off + h.numel()]
                off += h.numel()
            else:
                buf = torch.empty(h.numel(), dtype=h.dtype, device=self.z.device)  # compute stream's allocator pool
            if self.cuda:
                if ready is None:
                    ready = torch.cuda.Event()
                    ready.record(cur)
                rs = self.reload_stream
                with torch.cuda.stream(rs):
                    rs.wait_event(ready)
                    e = self.events.get((k, i))
                    if e is not None:
                        rs.wait_event(e)  # this chunk's offload has drained (and only this one)
                    buf.copy_(h, non_blocking=True)
                    buf.record_stream(rs)
                    ev = torch.cuda.Event()
                    ev.record(rs)
                self.events[(k, i)] = ev
            else:
                buf.copy_(h)
            self.tail[k][i] = buf
        if not self._pending():
            self.reloading = True
            self.n_reloads += 1

    def hosted(self, lo):
        """Does ``step()`` update the piece starting at ``lo`` on the host (host-step tails)?"""
        return (self.host_step and self.split and self.offloaded and lo >= self.a and "master" in self.host
                and all(k in self.host for k, v in self.z.store.states.items() if v is not None))

    def step_on_host(self, pieces, coef, lp_flat, found_inf=None, lp_cur=None):
        """Host Adam over the tail pieces [(lo, hi, group)]; the device kernels of the heads (already queued) run
        meanwhile. The bf16 parameters land in ``lp_flat``.

        ``found_inf`` (device flag: fp16 dynamic loss scaling, or a symmetric-memory skip) is the same skip the device
        kernels fold: when it is set the host tails are left untouched (and ``lp_flat``, if it is not the live
        parameter buffer ``lp_cur``, receives the current parameters of the pieces).

        On the GPU with ``lp_flat`` the live parameter buffer the host step is ASYNCHRONOUS (``async_host_step``):
        every tail gradient goes D2H at once (pieces in the order the next forward needs their units: the persistent
        root unit -- embeddings, LM head -- first, then the blocks in forward order), each piece's tail is zeroed on
        the copy stream right after its D2H, and a worker thread runs the host Adam piece by piece and issues each
        piece's bf16 H2D with its own event. ``step()`` returns at once; the next forward waits only for the pieces
        of the unit it is about to run (``wait_unit``), so the host Adam of the last blocks hides behind the forward
        of the first ones (reference stage3.py:2082-2144 overlaps the CPU step with the parameter swap-in the same
        way). Otherwise the pieces are stepped in place, D2H of piece i + 1 and H2D of piece i - 1 around the host
        update of piece i."""
        cur = torch.cuda.current_stream() if self.cuda else None
        if found_inf is not None and float(found_inf.reshape(-1)[0].item()) != 0.0:  # one sync, only when a flag exists
            if lp_cur is not None and lp_flat.data_ptr() != lp_cur.data_ptr():
                for lo, hi, _ in pieces:
                    lp_flat[lo:hi].copy_(lp_cur[lo:hi])
            self.host_skips = getattr(self, "host_skips", 0) + 1
            return
        coef = float(coef) if not torch.is_tensor(coef) else float(coef.item())
        if self.cuda and self.async_host_step and lp_cur is not None and lp_flat.data_ptr() == lp_cur.data_ptr():
            self._step_on_host_async(pieces, coef, lp_flat, cur)
        else:
            self._step_on_host_sync(pieces, coef, lp_flat, cur)
        self.host_steps = getattr(self, "host_steps", 0) + 1

    # async host step (GPU): see step_on_host
    async_host_step = os.environ.get("HDS_ASYNC_HOST_STEP", "1") == "1"

    def _adam_piece(self, lo, hi, g, grad, out, coef):
        from ...ops.cpu_optimizers import cpu_adam_flat
        z, s, a = self.z, self.z.store, self.a
        st = {k: self.host[k][lo - a:hi - a] for k in s.states if s.states[k] is not None}
        cpu_adam_flat(self.host["master"][lo - a:hi - a], grad, st["exp_avg"], st["exp_avg_sq"],
                      g["step"], g["lr"] * g.get("lr_mult", 1.0), tuple(g.get("betas", (0.9, 0.999))),
                      g.get("eps", 1e-8), g.get("weight_decay", 0.0), z.adamw, g.get("bias_correction", True),
                      bf16_out=out if out.dtype == torch.bfloat16 else None, grad_scale=coef)
        if out.dtype != torch.bfloat16:
            out.copy_(self.host["master"][lo - a:hi - a])

    def _forward_order(self, pieces):
        """Piece indices in the order the next forward reaches them: pieces of persistent (root) units first, then
        by the earliest forward position of any unit they overlap (the recorded trace, else store order)."""
        z = self.z
        trace = list(dict.fromkeys(getattr(z, "_fwd_trace", None) or []))
        pos = {uid: i for i, uid in enumerate(trace)}
        units = [(u.store_off, u.store_off + u.shard, -1 if u.persistent else pos.get(u.uid, len(pos) + u.uid))
                 for u in z.units if u.shard]

        def key(i):
            lo, hi, _ = pieces[i]
            ranks = [r for a0, b0, r in units if a0 < hi and lo < b0]
            return (min(ranks) if ranks else 1 << 30, lo)

        return sorted(range(len(pieces)), key=key)

    def _step_on_host_sync(self, pieces, coef, lp_flat, cur):
        s = self.z.store
        big = max(hi - lo for lo, hi, _ in pieces)
        if self._h_grad is None or self._h_grad[0].numel() < big:
            self._h_grad = [torch.empty(big, dtype=s.grad.dtype, pin_memory=self.cuda) for _ in range(2)]
            self._h_lp = [torch.empty(big, dtype=lp_flat.dtype, pin_memory=self.cuda) for _ in range(2)]
        d2h, h2d = [None, None], [None, None]

        def issue_d2h(i):
            lo, hi, _ = pieces[i]
            b = i & 1
            if not self.cuda:
                self._h_grad[b][:hi - lo].copy_(s.grad[lo:hi])
                return
            ev = torch.cuda.Event()
            ev.record(cur)
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                self._h_grad[b][:hi - lo].copy_(s.grad[lo:hi], non_blocking=True)
                d2h[b] = torch.cuda.Event()
                d2h[b].record(self.stream)

        issue_d2h(0)
        for i, (lo, hi, g) in enumerate(pieces):
            b, n = i & 1, hi - lo
            if i + 1 < len(pieces):
                issue_d2h(i + 1)
            if self.cuda:
                d2h[b].synchronize()
                if h2d[b] is not None:
                    h2d[b].synchronize()  # staging buffer b is free again
            out = self._h_lp[b][:n]
            self._adam_piece(lo, hi, g, self._h_grad[b][:n], out, coef)
            if self.cuda:
                with torch.cuda.stream(self.reload_stream):
                    lp_flat[lo:hi].copy_(out, non_blocking=True)
                    h2d[b] = torch.cuda.Event()
                    h2d[b].record(self.reload_stream)
            else:
                lp_flat[lo:hi].copy_(out)
        if self.cuda:
            cur.wait_stream(self.reload_stream)
            cur.wait_stream(self.stream)  # the gradient buffer is zeroed after step()

    def _step_on_host_async(self, pieces, coef, lp_flat, cur):
        import threading
        s, a = self.z.store, self.a
        n_tail = s.numel - a
        if self._h_grad_full is None or self._h_grad_full.numel() != n_tail or self._h_grad_full.dtype != s.grad.dtype:
            self._h_grad_full = torch.empty(n_tail, dtype=s.grad.dtype, pin_memory=True)
            self._h_lp_full = torch.empty(n_tail, dtype=lp_flat.dtype, pin_memory=True)
        order = self._forward_order(pieces)
        d2h = [None] * len(pieces)
        ev = torch.cuda.Event()
        ev.record(cur)
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            for i in order:
                lo, hi, _ = pieces[i]
                self._h_grad_full[lo - a:hi - a].copy_(s.grad[lo:hi], non_blocking=True)
                d2h[i] = torch.cuda.Event()
                d2h[i].record(self.stream)
                s.grad[lo:hi].zero_()  # the tail's zero_grad, behind its own D2H (zero_grad skips the tail)
            self._tail_grads_free = torch.cuda.Event()
            self._tail_grads_free.record(self.stream)
        ready = [threading.Event() for _ in pieces]
        h2d = [None] * len(pieces)
        dev = self.z.device
        self._async = {"pieces": pieces, "ready": ready, "h2d": h2d, "err": None}
        # unit -> the pieces it overlaps (the forward waits for exactly those)
        self._unit_pieces = {}
        for u in self.z.units:
            lo_u, hi_u = u.store_off, u.store_off + u.shard
            idx = [i for i, (lo, hi, _) in enumerate(pieces) if lo < hi_u and lo_u < hi]
            if idx:
                self._unit_pieces[u.uid] = idx
        rec = self._async

        def run():
            try:
                torch.cuda.set_device(dev)
                for i in order:
                    lo, hi, g = pieces[i]
                    d2h[i].synchronize()
                    out = self._h_lp_full[lo - a:hi - a]
                    self._adam_piece(lo, hi, g, self._h_grad_full[lo - a:hi - a], out, coef)
                    with torch.cuda.stream(self.reload_stream):
                        lp_flat[lo:hi].copy_(out, non_blocking=True)
                        e = torch.cuda.Event()
                        e.record(self.reload_stream)
                    h2d[i] = e
                    ready[i].set()
            except BaseException as e:  # noqa: BLE001 -- re-raised on the training thread at the next wait
                rec["err"] = e
                for r in ready:
                    r.set()

        self._thread = threading.Thread(target=run, name="hds-host-step", daemon=True)
        self._thread.start()
        self.async_steps = getattr(self, "async_steps", 0) + 1

    def _wait_pieces(self, idx, stream=None):
        rec = self._async
        if rec is None:
            return
        for i in idx:
            rec["ready"][i].wait()
            if rec["err"] is not None:
                raise RuntimeError("host-step optimizer thread failed") from rec["err"]
            e = rec["h2d"][i]
            if e is not None:
                (stream or torch.cuda.current_stream()).wait_event(e)

    def wait_unit(self, u):
        """Before unit ``u`` computes (its forward pre-hook, the root units at the forward start): order the current
        stream after the H2D of the host-stepped pieces holding its parameters."""
        if self._async is None:
            return
        idx = self._unit_pieces.pop(u.uid, None)
        if idx:
            self._wait_pieces(idx)
        if not self._unit_pieces:
            self.join()

    def before_backward(self):
        """The backward writes gradients into the tail: after the tail's D2H and zeroing (copy stream)."""
        ev = self.__dict__.pop("_tail_grads_free", None)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)

    def join(self):
        """Wait for the host-step thread (every piece issued) and order the current stream after all its H2D: before
        the next step, a checkpoint, or any reader of the host states."""
        t = self.__dict__.get("_thread")
        rec = self._async
        if t is not None:
            t.join()
            self._thread = None
        if rec is not None:
            self._async = None
            self._unit_pieces = {}
            if rec["err"] is not None:
                raise RuntimeError("host-step optimizer thread failed") from rec["err"]
            cur = torch.cuda.current_stream()
            for e in rec["h2d"]:
                if e is not None:
                    cur.wait_event(e)

    @property
    def async_pending(self):
        return self._async is not None

    def wait_tails(self):
        """Before ``step()``: every tail chunk on the device and ordered before the current stream (states stay
        split). Host-step tails stay where they are."""
        if not self.offloaded:
            return
        self.join()  # an async host step of the previous step must have issued every piece
        if self.host_step:
            return
        self.reload()
        if self.cuda:
            cur = torch.cuda.current_stream()
            for k in self.tail:
                for i in range(len(self.bounds)):
                    cur.wait_event(self.events[(k, i)])
        self.offloaded = False
        self.reloading = False

    def wait(self):
        """Whole flat states on the device (checkpoint save / load, fp32 fragment access): reload the tails and
        concatenate each state; they stay whole until the next step's ``offload()``."""
        self.join()
        if self.host_step and self.offloaded:
            self.reload()
            self.host_step, hs = False, True
            try:
                self.wait_tails()
            finally:
                self.host_step = hs
        else:
            self.wait_tails()
        if not self.split:
            return
        for k in list(self.tail):
            parts = self.tail.pop(k)
            head = self._get(k)
            self._set(k, torch.cat(([head] if head.numel() else []) + parts))
            del parts
        self.split = False

    ensure_resident = wait

    def on_backward_position(self, pos):
        if not self.offloaded or self.reloading or self.host_step:
            return
        if self.reload_pos is not None and pos is not None:  # placed by the compiled schedule (plan_state_reload)
            if pos <= self.reload_pos:
                self.reload()
            return
        if not self.cuda:
            self.reload()
            return
        # no schedule: bring the tails back as soon as the HBM the backward has freed holds all of them -- at the
        # start of backward when everything fits, later when the tails and the activations do not fit together;
        # step() reloads them if they never fit
        limit = int(self.mem_fraction * torch.cuda.get_device_properties(self.z.device).total_memory)
        alloc = torch.cuda.memory_allocated(self.z.device)
        pending = self._pending()
        if pending and alloc + sum(self._chunk_bytes(k, i) for k, i in pending) <= limit:
            self.reload(chunks=pending)  # all of it at once, in one allocation, as soon as it fits

    # HBM fraction the memory-driven reload may fill (HDS_STATE_RELOAD_FRACTION) and, without trace positions (one
    # rank), whether the backward reloads at all before step() (HDS_STATE_RELOAD_IN_BWD)
    mem_fraction = float(os.environ.get("HDS_STATE_RELOAD_FRACTION", "0.92"))
    untraced_backward_reload = os.environ.get("HDS_STATE_RELOAD_IN_BWD", "0") == "1"

    def stats(self):
        return {"state_bytes": self.bytes, "offloads": self.n_offloads, "reloads": self.n_reloads,
                "reload_pos": self.reload_pos, "ratio": self.ratio, "split_element": self.a,
                "chunks": len(self.bounds), "chunk_mb": round(self.chunk_bytes / 2**20, 3),
                "host_step": self.host_step, "host_steps": getattr(self, "host_steps", 0),
                "async_host_steps": getattr(self, "async_steps", 0),
                "fwd_waits": self.fwd_waits, "fwd_wait_s": round(self.fwd_wait_s, 3),
                **({"auto_ratio": self.auto_info} if self.auto_ratio else {}),
                "states": sorted(self.host) if self.host else sorted(self._keys())}
