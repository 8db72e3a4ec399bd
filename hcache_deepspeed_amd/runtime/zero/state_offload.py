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

Offload and reload run on SEPARATE copy streams: a reload issued while the post-step offload of other states is still
draining does not queue behind it -- it waits only for its own state's offload.
"""
import torch


class OptimizerStateOffload:

    def __init__(self, zopt, include_master=True, ratio=1.0):
        self.z = zopt
        self.include_master = bool(include_master)
        self.ratio = min(1.0, max(0.0, float(ratio)))
        dev = zopt.device
        self.cuda = dev.type == "cuda"
        self.stream = torch.cuda.Stream(dev, priority=-1) if self.cuda else None  # offload (D2H)
        self.reload_stream = torch.cuda.Stream(dev, priority=-1) if self.cuda else None  # reload (H2D)
        self.host = {}  # key -> pinned tail [n - a]
        self.tail = {}  # key -> device tail [n - a] while resident (reloaded), else absent
        self.events = {}  # key -> last D2H / H2D event of its tail
        self.split = False  # heads + tails (not whole flat states)
        self.offloaded = False  # tails off the device (not reloaded yet)
        self.reloading = False
        self.reload_pos = None  # backward trace position that triggers the reload (None: backward start)
        self.a = None  # split element
        self.bytes = 0
        self.n_offloads = 0
        self.n_reloads = 0

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

    def _split_at(self, n):
        if self.a is None:
            a = int(round((1.0 - self.ratio) * n))
            self.a = min(n, (a + 63) // 64 * 64) if a > 0 else 0  # 256-B aligned pieces for the vector kernels
        return self.a

    def cuts(self):
        """Element offsets at which ``step()`` must split its ranges (the head/tail boundary while split)."""
        return (self.a, ) if self.split and self.a else ()

    def view(self, k, lo, hi):
        """[lo, hi) of state ``k`` (``k`` = "master" or a moment key) inside ONE piece (never across a cut)."""
        if not self.split or k not in self.host:  # not split, or a state this executor does not move
            return self._get(k)[lo:hi]
        a = self.a
        if hi <= a:
            return self._get(k)[lo:hi]
        assert lo >= a, "a range across the head/tail cut"
        return self.tail[k][lo - a:hi - a]

    def moves(self, k):
        return k in self.host or (not self.split and k in self._keys())

    def state_bytes(self):
        """Bytes one offload moves each way."""
        if self.host:
            return sum(h.numel() * h.element_size() for h in self.host.values())
        n = self.z.store.numel
        return sum((n - self._split_at(n)) * self._get(k).element_size() for k in self._keys())

    # -----------------------------------------------------------------------------------------------------
    def offload(self):
        """After ``step()``: D2H every state's tail on the copy stream, release its HBM once the DMA drains. Whole
        (materialized) states are split first: the head is a new allocation, the whole buffer is released."""
        if self.offloaded:
            return
        self.bytes = 0
        cur = torch.cuda.current_stream() if self.cuda else None
        keys = self._keys() if not self.split else list(self.host)
        for k in keys:
            if self.split:
                t, head = self.tail.pop(k, None), None
                if t is None:
                    continue
            else:  # whole flat state -> head (stays) + tail (goes)
                full = self._get(k)
                n = full.numel()
                if n == 0:
                    continue
                a = self._split_at(n)
                head = full[:a].clone() if a else full.new_empty(0)
                t = full[a:]
            n_t = t.numel()
            h = self.host.get(k)
            if h is None or h.numel() != n_t:
                h = self.host[k] = torch.empty(n_t, dtype=t.dtype, pin_memory=self.cuda)
            if self.cuda:
                self.stream.wait_stream(cur)
                with torch.cuda.stream(self.stream):
                    h.copy_(t, non_blocking=True)
                    t.record_stream(self.stream)  # the block recycles only after the DMA drained
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                self.events[k] = ev
            else:
                h.copy_(t)
            if head is not None:
                self._set(k, head)
            self.bytes += n_t * t.element_size()
        self.split = True
        self.offloaded = True
        self.reloading = False
        self.n_offloads += 1

    def _pending(self):
        """(key, host tail) of the tails still off the device."""
        return [(k, h) for k, h in self.host.items() if k not in self.tail] if self.offloaded else []

    def reload(self, keys=None):
        """Issue the H2D of the offloaded tails (all, or ``keys``; non-blocking); ``wait_tails()`` orders the compute
        stream after it."""
        if not self.offloaded or self.reloading:
            return
        cur = torch.cuda.current_stream() if self.cuda else None
        for k, h in self._pending():
            if keys is not None and k not in keys:
                continue
            buf = torch.empty(h.numel(), dtype=h.dtype, device=self.z.device)  # compute stream's allocator pool
            if self.cuda:
                ready = torch.cuda.Event()
                ready.record(cur)
                rs = self.reload_stream
                with torch.cuda.stream(rs):
                    rs.wait_event(ready)
                    if k in self.events:
                        rs.wait_event(self.events[k])  # this tail's offload has drained (and only this one)
                    buf.copy_(h, non_blocking=True)
                    buf.record_stream(rs)
                    ev = torch.cuda.Event()
                    ev.record(rs)
                self.events[k] = ev
            else:
                buf.copy_(h)
            self.tail[k] = buf
        if not self._pending():
            self.reloading = True
            self.n_reloads += 1

    def wait_tails(self):
        """Before ``step()``: every tail on the device and ordered before the current stream (states stay split)."""
        if not self.offloaded:
            return
        self.reload()
        if self.cuda:
            cur = torch.cuda.current_stream()
            for k in self.tail:
                cur.wait_event(self.events[k])
        self.offloaded = False
        self.reloading = False

    def wait(self):
        """Whole flat states on the device (checkpoint save / load, fp32 fragment access): reload the tails and
        concatenate each state; they stay whole until the next step's ``offload()``."""
        self.wait_tails()
        if not self.split:
            return
        for k in list(self.tail):
            head, t = self._get(k), self.tail.pop(k)
            self._set(k, torch.cat([head, t]) if head.numel() else t)
        self.split = False

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
        # no schedule: bring each tail back as soon as the HBM the backward has freed holds it -- at the start of
        # backward when everything fits, late (tail by tail) when the tails and the activations do not fit
        # together; step() reloads whatever is left
        limit = int(self.mem_fraction * torch.cuda.get_device_properties(self.z.device).total_memory)
        for k, h in sorted(self._pending(), key=lambda x: -x[1].numel() * x[1].element_size()):
            if torch.cuda.memory_allocated(self.z.device) + h.numel() * h.element_size() <= limit:
                self.reload(keys={k})

    mem_fraction = 0.9

    def stats(self):
        return {"state_bytes": self.bytes, "offloads": self.n_offloads, "reloads": self.n_reloads,
                "reload_pos": self.reload_pos, "ratio": self.ratio, "split_element": self.a,
                "states": sorted(self.host) if self.host else sorted(self._keys())}
