"""Asynchronous optimizer-state offload between steps: the executor of DeepCompile's ``offload_adam_states`` pass.

Reference parity: compile/passes/offload_adam_states.py (offload tasks after the optimizer step on a copy stream,
per-key events, reload tasks placed in the backward graph so the states are back by the step) and
csrc/compile/z3.cpp:268-341 (dedicated offload / reload streams).

MI355X design: every state is ONE flat buffer of this rank's shard (runtime/zero/flat.py ``ShardStore``), so an
offload is one pinned-host DMA per state on a high-priority copy stream, issued right after ``step()`` and
overlapping the next forward; the device storage is released the moment its DMA drains (``record_stream`` +
``set_`` to an empty storage -- any stray access while offloaded sees a 0-element tensor and fails loudly instead
of reading stale data). The reload is issued at a backward trace position chosen by the pass
(``compile/passes.plan_state_reload``: the latest position whose remaining backward compute still covers the
measured H2D time) or, without a plan, state by state as soon as the HBM the backward has freed holds it; the device buffer is allocated on the compute stream
(whose allocator pool holds what backward freed) and ``step()`` waits on the per-state H2D events. Between those
two points the HBM the states occupied (12 B/param with the fp32 master) is free for activations.

Offload and reload run on SEPARATE copy streams (like the reference's dedicated streams in z3.cpp): a reload issued
while the post-step offload of other states is still draining does not queue behind it -- it waits only for its own
state's offload. ``ratio`` < 1 offloads only that fraction of the state bytes (whole states, the largest first): the
partial offload for a model whose states almost fit, planned from the bytes the step is over budget.
"""
import torch


class OptimizerStateOffload:

    def __init__(self, zopt, include_master=True, ratio=1.0):
        self.z = zopt
        self.include_master = bool(include_master)
        self.ratio = float(ratio)
        dev = zopt.device
        self.cuda = dev.type == "cuda"
        self.stream = torch.cuda.Stream(dev, priority=-1) if self.cuda else None  # offload (D2H)
        self.reload_stream = torch.cuda.Stream(dev, priority=-1) if self.cuda else None  # reload (H2D)
        self.host = {}
        self.events = {}
        self.offloaded = False
        self.reloading = False
        self.reload_pos = None  # backward trace position that triggers the reload (None: backward start)
        self.bytes = 0
        self.n_offloads = 0
        self.n_reloads = 0

    def _tensors(self):
        """Device-resident states this executor moves (host-resident ones -- ZeRO-Offload -- are left alone; an
        fp32 master that IS the compute-dtype shard, as in fp32 training, stays too); with ``ratio`` < 1 the largest
        states first, until that fraction of their bytes is covered."""
        s = self.z.store
        out = [(k, v) for k, v in s.states.items() if v is not None and v.device.type == self.z.device.type]
        m = s.master
        if (self.include_master and m is not None and m.device.type == self.z.device.type
                and not (m.numel() and s.lp.numel() and m.data_ptr() == s.lp.data_ptr())):
            out.append(("master", m))
        if self.ratio < 1.0:
            if not hasattr(self, "_keys"):  # fixed at the first call (sizes never change; offloaded ones read 0)
                size = lambda kv: kv[1].numel() * kv[1].element_size()  # noqa: E731
                total = sum(size(kv) for kv in out)
                keys, acc = [], 0
                for kv in sorted(out, key=size, reverse=True):
                    if acc >= self.ratio * total - 1:
                        break
                    keys.append(kv[0])
                    acc += size(kv)
                self._keys = set(keys)
            out = [kv for kv in out if kv[0] in self._keys]
        return out

    def state_bytes(self):
        return sum(self.host[k].numel() * self.host[k].element_size() for k in self.host) if self.host else \
            sum(t.numel() * t.element_size() for _, t in self._tensors())

    # -----------------------------------------------------------------------------------------------------
    def offload(self):
        """After ``step()``: D2H every state on the copy stream, release its HBM once the DMA drains."""
        if self.offloaded:
            return
        self.bytes = 0
        cur = torch.cuda.current_stream() if self.cuda else None
        for k, t in self._tensors():
            n = t.numel()
            if n == 0:
                continue
            h = self.host.get(k)
            if h is None or h.numel() != n:
                h = self.host[k] = torch.empty(n, dtype=t.dtype, pin_memory=self.cuda)
            if self.cuda:
                self.stream.wait_stream(cur)
                with torch.cuda.stream(self.stream):
                    h.copy_(t.view(-1), non_blocking=True)
                    t.record_stream(self.stream)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                self.events[k] = ev
            else:
                h.copy_(t.view(-1))
            t.set_(torch.empty(0, dtype=t.dtype, device=t.device))
            self.bytes += n * t.element_size()
        self.offloaded = True
        self.reloading = False
        self.n_offloads += 1

    def _pending(self):
        """(key, tensor, host) of the states still off the device."""
        return [(k, t, self.host[k]) for k, t in self._tensors() if k in self.host and t.numel() == 0]

    def reload(self, keys=None):
        """Issue the H2D of the offloaded states (all, or ``keys``; non-blocking); ``wait()`` orders the compute
        stream after it."""
        if not self.offloaded or self.reloading:
            return
        cur = torch.cuda.current_stream() if self.cuda else None
        for k, t in self._tensors():
            h = self.host.get(k)
            if h is None or t.numel() != 0 or (keys is not None and k not in keys):
                continue
            buf = torch.empty(h.numel(), dtype=h.dtype, device=t.device)  # compute stream's allocator pool
            if self.cuda:
                ready = torch.cuda.Event()
                ready.record(cur)
                rs = self.reload_stream
                with torch.cuda.stream(rs):
                    rs.wait_event(ready)
                    if k in self.events:
                        rs.wait_event(self.events[k])  # this state's offload has drained (and only this one)
                    buf.copy_(h, non_blocking=True)
                    buf.record_stream(rs)
                    ev = torch.cuda.Event()
                    ev.record(rs)
                self.events[k] = ev
            else:
                buf.copy_(h)
            t.set_(buf)
        if not self._pending():
            self.reloading = True
            self.n_reloads += 1

    def wait(self):
        """Make the states usable on the current stream (reloading first if nothing scheduled it)."""
        if not self.offloaded:
            return
        self.reload()
        if self.cuda:
            cur = torch.cuda.current_stream()
            for ev in self.events.values():
                cur.wait_event(ev)
        self.offloaded = False
        self.reloading = False

    ensure_resident = wait

    def on_backward_position(self, pos):
        if not self.offloaded or self.reloading:
            return
        if self.reload_pos is not None:  # placed by the compiled schedule (compile/passes.plan_state_reload)
            if pos is not None and pos <= self.reload_pos:
                self.reload()
            return
        if not self.cuda:
            self.reload()
            return
        # no schedule: bring each state back as soon as the HBM the backward has freed holds it -- at the start of
        # backward when everything fits, late (state by state) when the states and the activations do not fit
        # together; step() reloads whatever is left
        limit = int(self.mem_fraction * torch.cuda.get_device_properties(self.z.device).total_memory)
        for k, t, h in sorted(self._pending(), key=lambda x: -x[2].numel() * x[2].element_size()):
            if torch.cuda.memory_allocated(self.z.device) + h.numel() * h.element_size() <= limit:
                self.reload(keys={k})

    mem_fraction = 0.9

    def stats(self):
        return {"state_bytes": self.bytes, "offloads": self.n_offloads, "reloads": self.n_reloads,
                "reload_pos": self.reload_pos, "ratio": self.ratio,
                "states": sorted(k for k, _ in self._tensors()) if self.ratio < 1.0 else "all"}
