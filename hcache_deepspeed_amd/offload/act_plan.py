"""Per-tensor activation plan (host activation cache policy ``"plan"``): every saved activation of a transformer block
is KEPT in HBM, SPILLED to pinned host memory (D2H on the copy stream in forward, prefetched H2D in backward), or
RECOMPUTED in backward from the tensors it was derived from -- decided per (block, tensor class).

Why per tensor and not per block (BASELINE config 3, Llama-3-8B at 32k tokens): a block saves ~4.6 GB whose costs
differ by two orders of magnitude per byte. Recomputing the whole block (activation checkpointing) spends ~27 ms to
free ~4.3 GB, 40 % of it re-running FlashAttention, whose output and LSE are only 6 % of the bytes. Per class:

=========================  =========  =====================================  ==========
class (Llama block)        bytes      recomputed from                        ms per GB
=========================  =========  =====================================  ==========
``norm_out`` x1, x2        268 MB x2  the saved pre-norm residual (1 pass)   ~0.6
``glu_t`` (hT)             940 MB     the saved gate|up output (1 pass)      ~0.6
``linear_out`` (gate|up)   1.88 GB    x2 @ W_gu (GEMM)                       ~2.7
``qkv``                    403 MB     RoPE(x1 @ W_qkv)                       ~2.9
``resid`` h2               268 MB     o @ W_o + h1                           ~2.7
``attn_out``, ``attn_lse`` 272 MB     FlashAttention forward                 ~40
=========================  =========  =====================================  ==========

so the plan recomputes the cheap-per-byte classes, spills the expensive ones over PCIe as far as the copy stream can
hide them inside the forward, and keeps the rest; block-level recompute is never the cheapest option.

Mechanism:

* **op tags** -- while a planned cache's forward runs, ops declare the class of their outputs and, optionally, a
  recipe ``fn(*srcs)`` that recomputes the output from other tensors (``tag``): the norm (its output from the saved
  pre-norm sum; the pre-norm sum as an add), the ZeRO linear (its output as ``x @ W^T``), attention (RoPE composed
  onto the qkv projection's recipe; o and LSE carry no recipe), SwiGLU (its transposed output from the gate|up
  tensor). Tags live in a per-forward registry keyed by the tensor's base object (weakly referenced, so a dead
  tensor's entry goes with it) and are consumed when the tensor is packed.
* **pack** (``saved_tensors_hooks``) -- a saved tensor of a tracked block becomes a reference to one handle per base
  tensor (views and repeated saves of the same tensor share it: the attention output saved by FlashAttention and by
  the O projection is spilled once). Recipe sources resolve to the handles of tensors saved earlier; sources that
  are never saved but carry a recipe (the O projection output inside h2 = o W_o + h1) are inlined. The action comes
  from the plan for (block, class).
* **unpack** -- KEEP returns the tensor, SPILL waits for the prefetch (started, as in the base cache, when backward
  first touches a later block), RECOMPUTE runs the recipe on the compute stream (sources unpacked recursively, the
  block's ZeRO-3 unit is gathered at that point). Each handle counts its consumers and drops its device / host
  memory after the last one.
* **plan** (``plan_tensors``) -- from a calibration step that spills everything: bytes per (block, class), the peak
  with everything spilled, per-class recipe time (each recipe run once with HIP events), and the PCIe rate as bytes
  over copy-BUSY time (per-copy events; the first-to-last span of the ``auto`` policy included idle gaps and read
  4x low). The over-budget bytes are freed by the cheapest options per byte: recomputing classes whose recipe costs
  less than a spill, then spilling (earliest blocks first, the classes most expensive to recompute first) up to the
  bytes the copy stream drains within ``spill_overlap`` of the forward time measured on the first planned step,
  then recomputing by cost per byte. After every step the measured forward/backward turn-around peak corrects the
  base estimate, the forward time against the no-spill forward measures what the spills really cost (concurrent
  copies slow the kernels they overlap; a spill whose memory the allocator must wait for stalls it), a step that
  slowed by more than twice the modelled cost backs the spill capacity off by a quarter, and the plan is recomputed
  (closed loop).

Reference anchors: FPDT's host chunk spill (sequence/fpdt_layer.py:462-508), CPU activation checkpointing
(runtime/activation_checkpointing/checkpointing.py:474-486), the DeepCompile offload_activation pass
(compile/passes/offload_activation.py:43-110).
"""
import contextlib
import weakref

import torch

from ..utils.logging import log_dist
from .activation_cache import HostActivationCache, _Spilled, default_host_budget_gib
from ..ops.hostcopy import d2h_
from .pinned import PinnedPool

KEEP, SPILL, RECOMPUTE = "keep", "spill", "recompute"

# -------------------------------------------------------------------------------------------------------------------
# op-side tag registry
# -------------------------------------------------------------------------------------------------------------------
_ACTIVE = None  # the PlannedActivationCache whose forward is running; ops tag only then


class _Tag:
    __slots__ = ("ref", "kind", "fn", "srcs", "__weakref__")

    def __init__(self, ref, kind, fn, srcs):
        self.ref, self.kind, self.fn, self.srcs = ref, kind, fn, srcs


def _base(t):
    return t._base if t._base is not None else t


def tracking():
    """True inside a planned cache's forward (custom Functions run their forward with grad mode off, so this does not
    look at grad mode)."""
    return _ACTIVE is not None


def tag(t, kind, fn=None, srcs=()):
    """Declare op output ``t``'s activation class ``kind`` and, optionally, a recipe: ``fn(*srcs)`` returns a tensor
    equal to ``t``'s base (``srcs``: tensors -- resolved to saved activations when ``t`` is packed -- or constants,
    e.g. Parameters, whose ``.data`` the ZeRO-3 backward gather has refreshed). No-op outside a planned forward."""
    c = _ACTIVE
    if c is None or not torch.is_tensor(t):
        return
    b = _base(t)
    key = id(b)
    reg = c._tags
    reg[key] = _Tag(weakref.ref(b, lambda _r, k=key, reg=reg: reg.pop(k, None)), kind, fn, tuple(srcs))


def lookup(t):
    """The tag of ``t``'s base tensor, or None."""
    c = _ACTIVE
    if c is None or not torch.is_tensor(t):
        return None
    b = _base(t)
    e = c._tags.get(id(b))
    return e if e is not None and e.ref() is b else None


# -------------------------------------------------------------------------------------------------------------------
# handles
# -------------------------------------------------------------------------------------------------------------------
class _Handle(_Spilled):
    """One saved base tensor of a tracked block (see module docstring). Inherits the spill fields (host buffer,
    events, prefetched device copy) so the base cache's prefetch machinery drives SPILL handles."""
    __slots__ = ("cls", "nbytes", "action", "t", "fn", "srcs", "refs", "stride", "saved")

    def __init__(self, layer, cls, nbytes, action):
        super().__init__()
        self.layer, self.cls, self.nbytes, self.action = layer, cls, nbytes, action
        self.host = None
        self.t = None
        self.fn, self.srcs = None, ()
        self.refs = 0
        self.saved = True


class _Ref:
    """What a pack returns: a handle plus the saved tensor's geometry inside the handle's base."""
    __slots__ = ("h", "shape", "stride", "offset")

    def __init__(self, h, t, base):
        self.h = h
        self.shape, self.stride = tuple(t.shape), tuple(t.stride())
        self.offset = t.storage_offset() - base.storage_offset()

    def view_of(self, base):
        if self.offset == 0 and self.shape == tuple(base.shape) and self.stride == tuple(base.stride()):
            return base
        return base.as_strided(self.shape, self.stride, base.storage_offset() + self.offset)


# -------------------------------------------------------------------------------------------------------------------
# planner (pure; unit-tested on CPU)
# -------------------------------------------------------------------------------------------------------------------
def plan_tensors(items, peak_all, budget, rec_ms, spill_cap_bytes, spill_ms_per_gb=0.6, no_spill_layers=(),
                 margin=1 << 30):
    """Choose an action per (layer, cls).

    items: {(layer, cls): bytes}; peak_all: the step peak with every item off the device; budget: HBM bytes;
    rec_ms: {cls: ms to recompute one item} (missing / None: not recomputable); spill_cap_bytes: bytes the copy
    stream can hide per step; spill_ms_per_gb: the (small) cost of a hidden spill -- concurrent kernels slow down
    while a copy runs. Returns ({(layer, cls): action}, estimated ms of added compute).
    """
    actions = {k: KEEP for k in items}
    need = peak_all + sum(items.values()) - (budget - margin)
    if need <= 0:
        return actions, 0.0
    no_spill = set(no_spill_layers)

    def per_gb(c, b):
        r = rec_ms.get(c)
        return None if r is None else r / max(b / 1e9, 1e-9)

    cands = []  # (cost per GB, order, action, key)
    for (l, c), b in items.items():
        r = per_gb(c, b)
        if r is not None:
            cands.append((r, l, RECOMPUTE, (l, c)))
        if l not in no_spill:
            # among equal spill costs: earliest block first (its D2H has the whole forward left to drain, its H2D the
            # whole backward), then the class most expensive to recompute (not recomputable = infinitely so)
            cands.append((spill_ms_per_gb, (l, -(r if r is not None else float("inf"))), SPILL, (l, c)))
    cands.sort(key=lambda x: (x[0], x[1] if isinstance(x[1], tuple) else (x[1], 0.0)))
    spilled = 0
    cost = 0.0
    for c_gb, _, act, key in cands:
        if need <= 0:
            break
        if actions[key] != KEEP:
            continue
        b = items[key]
        if act == SPILL:
            if spilled + b > spill_cap_bytes:
                continue
            spilled += b
        actions[key] = act
        cost += c_gb * b / 1e9
        need -= b
    return actions, cost


# -------------------------------------------------------------------------------------------------------------------
# the cache
# -------------------------------------------------------------------------------------------------------------------
class PlannedActivationCache(HostActivationCache):
    """Host activation cache with a per-tensor keep / spill / recompute plan (policy ``"plan"``).

    ``forced``: optional {cls: action} applied to every tracked block without calibration (tests, experiments)."""

    def __init__(self, device, spill_cost_ms_per_gb=0.6, forced=None, **kw):
        kw.setdefault("spill_overlap", 0.8)
        super().__init__(device, **kw)
        self.spill_cost = float(spill_cost_ms_per_gb)
        self.forced = dict(forced) if forced else None
        self._tags = {}
        self._handles = {}  # id(base) -> (weakref(base), handle) for this forward's saved tensors
        self._occ = {}  # (layer, kind) -> next occurrence index
        self.actions = None  # {(layer, cls): action}
        self.items = {}  # {(layer, cls): bytes} measured by the calibration step
        self.rec_ms = {}  # {cls: ms}
        self._rec_timed = set()
        self._peak_all = None
        self._stage = 0  # 0 calibrate next, 1 calibrating, 2 first planned step (timed forward), 3 closed loop
        self._copy_busy = [0.0, 0]  # ms, bytes of timed calibration copies
        self._copy_evs = []
        self.t_fwd_ms = None
        self.spill_cost_measured = None  # ms per spilled GB the forward actually slowed down by (EMA, reported)
        self.cap_scale = 1.0  # fraction of the PCIe-time spill capacity the plan may use (backed off when measured)
        self.est_cost_ms = 0.0
        self.step_spill_bytes = 0
        self.step_recomputed = 0
        self._spill_acc = 0
        self._rec_acc = 0
        self.replans = 0
        self._cal_items, self._cal_kept, self._rec_candidates = {}, 0, {}

    @classmethod
    def from_config(cls, cfg, device):
        budget = None
        if device.type == "cuda":
            gib = float(getattr(cfg, "gpu_budget_gib", 0.0) or 0.0)
            total = torch.cuda.get_device_properties(device).total_memory
            budget = int(gib * 2**30) if gib > 0 else int(0.92 * total)
        hgib = float(getattr(cfg, "host_budget_gib", 0.0) or 0.0)
        if hgib <= 0:
            hgib = default_host_budget_gib()
        wgib = float(getattr(cfg, "copy_window_gib", 0.0) or 0.0)
        return cls(device, spill_cost_ms_per_gb=float(getattr(cfg, "spill_cost_ms_per_gb", 0.6)),
                   forced=getattr(cfg, "forced_actions", None),
                   min_bytes=1 << 20, min_layers_resident=cfg.min_layers_resident,
                   prefetch_layers=int(getattr(cfg, "prefetch_layers", 2)), gpu_budget_bytes=budget,
                   host_budget_bytes=int(hgib * 2**30), copy_window_bytes=int(wgib * 2**30) if wgib > 0 else None,
                   spill_overlap=float(getattr(cfg, "spill_overlap", 0.8)))

    def attach(self, model):
        # tracking only: recomputation is per tensor (recipes), not per block -- no block wrappers
        rec, ck = self.policy_recompute, self.ckpt_offload
        self.policy_recompute = self.ckpt_offload = False
        try:
            return super().attach(model)
        finally:
            self.policy_recompute, self.ckpt_offload = rec, ck

    # ---------------------------------------------------------------------------------------------------------------
    def _action(self, layer, cls):
        if self.forced is not None:
            return self.forced.get(cls, KEEP)
        if self._stage <= 1:  # calibrating: everything off the device (the base cache's calibration)
            return KEEP if layer >= self.n_layers - self.keep else SPILL
        return self.actions.get((layer, cls), KEEP)

    @contextlib.contextmanager
    def forward_context(self):
        global _ACTIVE
        cuda = self.device.type == "cuda"
        self._end_of_step()
        if cuda:
            self._take_step_peak()  # the previous step's full peak, across the per-block resets of its backward
        if cuda and self.forced is None and self.budget is not None:
            self._advance_plan()
            self._turn_peak = None
        if cuda:
            torch.cuda.reset_peak_memory_stats(self.device)
        self.cur_layer = -1
        self._release_stale()
        self.by_layer = {}
        self.layer_bytes = {}
        self._capped_this_step = 0
        self._bwd_layer, self._bwd_mark = None, None
        self._handles, self._occ, self._tags = {}, {}, {}
        timed = cuda and self._stage >= 2 and self.forced is None
        if timed:
            self._fwd_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self._fwd_ev[0].record()
        prev, _ACTIVE = _ACTIVE, self
        try:
            with torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack):
                yield
        finally:
            _ACTIVE = prev
            self._tags = {}
            self._handles = {}
        if timed:
            self._fwd_ev[1].record()
        if cuda and self._turn_peak is None:
            self._turn_peak = torch.cuda.max_memory_allocated(self.device)

    def _was_calibrating(self):
        return self._stage == 1

    def _end_of_step(self):
        self.step_spill_bytes, self.step_recomputed = self._spill_acc, self._rec_acc
        self._spill_acc = self._rec_acc = 0

    def _release_stale(self):
        for lst in self.by_layer.values():  # a forward whose backward never ran: return its host buffers
            for o in lst:
                if o.dev is not None and o.h2d_done is not None:
                    torch.cuda.current_stream().wait_event(o.h2d_done)
                o.dev = None
                if o.host is not None:
                    if o.h2d_done is not None and self.stream is not None:
                        self.stream.wait_event(o.h2d_done)
                    if self.device.type == "cuda":
                        self.host_in_use -= PinnedPool.nbytes_of(o.host)
                        self.pool.put(o.host)
                    o.host = None

    def _advance_plan(self):
        if self._stage == 0:
            self._stage = 1  # this forward calibrates
            self._cal_items, self._cal_kept, self._rec_candidates = {}, 0, {}
            return
        if self._stage == 1:
            # the peak with every item off the device: the measured one minus what calibration kept (the last
            # blocks, and tensors the pinned-host cap left on the GPU)
            self._peak_all = self.last_step_peak - self._cal_kept
            ms, nb = self._copy_busy
            for a, b, n in self._copy_evs:
                b.synchronize()
                ms += a.elapsed_time(b)
                nb += n
            self._copy_evs = []
            self.pcie_gbps = nb / ms / 1e6 if ms > 0 else None
            self.items = dict(self._cal_items)
            # first planned step: no spilling yet (the forward it times sets the spill capacity)
            self._replan(spill_cap=0)
            self._stage = 2
            return
        t_last = None
        if self._fwd_ev is not None:
            s, e = self._fwd_ev
            e.synchronize()  # the forward ended a whole backward ago
            t_last = s.elapsed_time(e)
            self._fwd_ev = None
        if self._stage == 2 and t_last is not None:
            self.t_fwd_ms = t_last  # forward with no spills: the base of the spill capacity and the spill cost
            self._stage = 3
        elif t_last is not None and self.step_spill_bytes > (1 << 30) and self.t_fwd_ms:
            # what spilling actually cost: the copies slow the kernels they overlap (measured, not modelled). The
            # cost is not linear in the bytes -- ~0 while the copies hide behind the forward, growing once they do
            # not (or once the allocator waits on a spill's copy for its memory) -- so a step whose forward slowed
            # by more than twice the modelled cost backs the spill CAPACITY off by a quarter instead of pricing every
            # spilled GB higher (which would switch spilling off for good on one slow sample).
            meas = max(0.0, t_last - self.t_fwd_ms) / (self.step_spill_bytes / 1e9)
            self.spill_cost_measured = meas if self.spill_cost_measured is None else \
                0.5 * (self.spill_cost_measured + meas)
            if meas > 2 * self.spill_cost:
                self.cap_scale = max(0.25, 0.75 * self.cap_scale)
        elif t_last is not None and self.step_spill_bytes <= (1 << 30) and self.t_fwd_ms:
            self.t_fwd_ms = min(self.t_fwd_ms, t_last)  # a no-spill forward refines the base
        if self._turn_peak is not None:
            # closed loop: the measured turn-around peak corrects the all-off-device base estimate
            kept = sum(b for k, b in self.items.items() if self.actions.get(k, KEEP) == KEEP)
            err = self._turn_peak - (self._peak_all + kept)
            if self.replans == 0 or err > 0 or err < -(2 << 30):
                self._peak_all += err
        self._replan()

    def spill_capacity(self):
        if not self.pcie_gbps or not self.t_fwd_ms:
            return 0
        return int(self.cap_scale * self.spill_overlap * self.t_fwd_ms * 1e-3 * self.pcie_gbps * 1e9)

    def _replan(self, spill_cap=None):
        cap = self.spill_capacity() if spill_cap is None else spill_cap
        no_spill = range(self.n_layers - self.keep, self.n_layers)
        cost = self.spill_cost
        new, self.est_cost_ms = plan_tensors(self.items, self._peak_all, self.plan_budget(), self.rec_ms, cap, cost,
                                             no_spill)
        if new != self.actions:
            self.replans += 1
            n = {a: sum(1 for v in new.values() if v == a) for a in (KEEP, SPILL, RECOMPUTE)}
            sb = sum(b for k, b in self.items.items() if new[k] == SPILL)
            rb = sum(b for k, b in self.items.items() if new[k] == RECOMPUTE)
            log_dist(f"activation plan: keep {n[KEEP]}, spill {n[SPILL]} ({sb / 2**30:.1f} GiB, cap "
                     f"{cap / 2**30:.1f} GiB), recompute {n[RECOMPUTE]} ({rb / 2**30:.1f} GiB, ~{self.est_cost_ms:.0f} ms)"
                     f" | base peak {self._peak_all / 2**30:.1f} GiB, budget {self.budget / 2**30:.1f} GiB, PCIe "
                     f"{(self.pcie_gbps or 0):.1f} GB/s busy-rate, forward {self.t_fwd_ms or 0:.0f} ms, spill cost "
                     f"{cost:.2f} ms/GB", ranks=[0])
        self.actions = new

    # ---------------------------------------------------------------------------------------------------------------
    def _cls(self, layer, kind):
        k = (layer, kind)
        i = self._occ.get(k, 0)
        self._occ[k] = i + 1
        return f"{kind}#{i}"

    def _find(self, b):
        e = self._handles.get(id(b))
        return e[1] if e is not None and e[0]() is b else None

    def _resolve(self, src, depth=0):
        """A recipe source -> ("ref", _Ref) | ("const", value) | None (unresolvable)."""
        if not torch.is_tensor(src):
            return ("const", src)
        if isinstance(src, torch.nn.Parameter) or (src.is_leaf and not src.requires_grad):
            return ("const", src)
        b = _base(src)
        h = self._find(b)
        if h is not None:
            return ("ref", _Ref(h, src, b))
        e = lookup(src)
        if e is None or e.fn is None or depth > 4:
            return None
        srcs = [self._resolve(s, depth + 1) for s in e.srcs]
        if any(s is None for s in srcs):
            return None
        h = _Handle(self.cur_layer, "inline", 0, RECOMPUTE)  # never saved: recomputed for its one consumer
        h.fn, h.srcs, h.saved = e.fn, srcs, False
        self._tags.pop(id(b), None)
        return ("ref", _Ref(h, src, b))

    def _pack(self, t):
        if (not isinstance(t, torch.Tensor) or self.cur_layer < 0 or t.numel() * t.element_size() < self.min_bytes
                or (self.device.type == "cuda" and not t.is_cuda)):
            return t
        layer = self.cur_layer
        b = _base(t)
        h = self._find(b)
        if h is not None:  # another save of the same tensor (a view, or a second consumer): share its handle
            h.refs += 1
            return _Ref(h, t, b)
        e = lookup(t)
        if b.is_leaf and e is None:
            # parameters and long-lived constants (RoPE tables); tensors an op created inside its forward are leaves
            # at pack time too, but those carry a tag
            return t
        cls = self._cls(layer, e.kind if e is not None else "other")
        nbytes = b.numel() * b.element_size()
        if not b.is_contiguous():
            return t  # outside the plan (kept as is)
        srcs = None
        if e is not None and e.fn is not None:
            srcs = [self._resolve(s) for s in e.srcs]
            if any(s is None for s in srcs):
                srcs = None
        self._tags.pop(id(_base(t)), None)
        if self._stage == 1 and self.forced is None:
            self._cal_items[(layer, cls)] = self._cal_items.get((layer, cls), 0) + nbytes
            if srcs is not None and cls not in self._rec_timed:
                self._rec_candidates[cls] = (e.fn, srcs)
        act = self._action(layer, cls)
        if act == RECOMPUTE and srcs is None:
            act = KEEP  # no usable recipe for this instance
        if act == SPILL and self.host_budget is not None and self.host_in_use + nbytes > self.host_budget:
            self.host_capped_bytes += nbytes
            self._capped_this_step += nbytes
            act = KEEP
        if self._stage == 1 and act != SPILL:
            self._cal_kept += nbytes
        h = _Handle(layer, cls, nbytes, act)
        h.refs = 1
        self._handles[id(b)] = (weakref.ref(b), h)
        if act == KEEP:
            h.t = b
        elif act == RECOMPUTE:
            h.fn, h.srcs = e.fn, srcs
            self._count_srcs(srcs)
            self._rec_acc += 1
        else:
            self._spill_to_host(h, b)
            self._spill_acc += nbytes
        return _Ref(h, t, b)

    def _count_srcs(self, srcs):
        """A recipe that will run consumes each source once; an inlined (never saved) source's recipe consumes its own
        sources in turn."""
        for kind, s in srcs:
            if kind == "ref":
                s.h.refs += 1
                if not s.h.saved:
                    self._count_srcs(s.h.srcs)

    def _spill_to_host(self, h, b):
        h.shape, h.dtype, h.device = b.shape, b.dtype, b.device
        nbytes = h.nbytes
        self.layer_bytes[h.layer] = self.layer_bytes.get(h.layer, 0) + nbytes
        if self.device.type != "cuda":  # CPU: a plain copy stands in for the host tier (tests)
            h.host = b.detach().clone().view(-1)
            self.by_layer.setdefault(h.layer, []).append(h)
            self.bytes_offloaded += nbytes
            return
        self._window(self._d2h_q, nbytes)
        h.host = self.pool.get(b.numel(), b.dtype)
        ev = torch.cuda.Event()
        ev.record()
        timed = self._stage == 1
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(self.stream)
            d2h_(h.host, b.view(-1))  # few-workgroup copy kernel, not the wide blit (ops/hostcopy.py)
            b.record_stream(self.stream)
            h.d2h_done = torch.cuda.Event(enable_timing=timed)
            h.d2h_done.record(self.stream)
            if timed:
                self._copy_evs.append((e0, h.d2h_done, nbytes))
        self._d2h_q.append((h.d2h_done, nbytes))
        self.bytes_offloaded += nbytes
        self.host_in_use += PinnedPool.nbytes_of(h.host)
        self.by_layer.setdefault(h.layer, []).append(h)

    def _prefetch(self, s):
        if self.device.type != "cuda":
            if s.dev is None and s.host is not None:
                s.dev = s.host.view(s.shape)
            return
        super()._prefetch(s)

    # ---------------------------------------------------------------------------------------------------------------
    def _value(self, h, consume=True):
        """The base tensor of handle ``h`` (materialised if needed); ``consume`` counts one consumer."""
        if h.action == KEEP:
            v = h.t
        elif h.action == SPILL:
            if h.dev is None:
                if h.host is None:
                    raise RuntimeError(f"activation plan: spilled {h.cls} of block {h.layer} unpacked after release")
                if self._stage != 1:  # (calibration times recipes on sources nobody prefetched yet)
                    self.late_unpacks += 1
                self._prefetch(h)
            if h.h2d_done is not None:
                torch.cuda.current_stream().wait_event(h.h2d_done)
            v = h.dev
        else:
            v = h.t
            if v is None:
                # a peek (consume=False: calibration timing) must not consume the sources either, nor cache
                args = [self._src_value(s, consume) for s in h.srcs]
                with torch.no_grad():
                    v = h.fn(*args)
                if consume:
                    h.t = v
        if consume:
            h.refs -= 1
            if h.refs <= 0:
                self._release(h)
        return v

    def _src_value(self, s, consume=True):
        kind, x = s
        if kind == "const":
            return x
        return x.view_of(self._value(x.h, consume))

    def _release(self, h):
        h.t = None
        if h.action == SPILL:
            h.dev = None
            if h.host is not None:
                if self.device.type == "cuda":
                    self.host_in_use -= PinnedPool.nbytes_of(h.host)
                    self.pool.put(h.host)
                h.host = None

    def _unpack(self, r):
        if not isinstance(r, _Ref):
            return r
        h = r.h
        self._prefetch_before(h.layer)
        if self._stage == 1 and self._rec_candidates:
            self._time_recipes()
        return r.view_of(self._value(h))

    def _time_recipes(self):
        """Calibration backward: run each class's recipe once (sources materialised first) and time it."""
        cuda = self.device.type == "cuda"
        for cls, (fn, srcs) in list(self._rec_candidates.items()):
            self._rec_timed.add(cls)
            try:
                args = [self._src_value(s, consume=False) for s in srcs]
            except RuntimeError:
                continue  # a source was already released: leave the class unrecomputable for now
            if cuda:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            with torch.no_grad():
                fn(*args)
            if cuda:
                e1.record()
                e1.synchronize()
                self.rec_ms[cls] = e0.elapsed_time(e1)
            else:
                self.rec_ms[cls] = 1.0
        self._rec_candidates = {}

    def stats(self):
        s = super().stats()
        acts = self.actions or {}
        s.update({"policy": "plan", "spill_bytes_step": self.step_spill_bytes,
                  "spill_gib_planned": round(sum(b for k, b in self.items.items() if acts.get(k) == SPILL) / 2**30, 2),
                  "recompute_gib_planned": round(sum(b for k, b in self.items.items() if acts.get(k) == RECOMPUTE)
                                                 / 2**30, 2),
                  "recomputed_tensors_step": self.step_recomputed, "est_recompute_ms": round(self.est_cost_ms, 1),
                  "recipe_ms": {k: round(v, 3) for k, v in sorted(self.rec_ms.items())},
                  "t_fwd_ms": None if self.t_fwd_ms is None else round(self.t_fwd_ms, 1),
                  "spill_cost_ms_per_gb": round(self.spill_cost, 3), "spill_cap_scale": round(self.cap_scale, 3),
                  "spill_cost_measured": None if self.spill_cost_measured is None else
                  round(self.spill_cost_measured, 3),
                  "spill_cap_gib": round(self.spill_capacity() / 2**30, 1), "replans": self.replans,
                  "spilled_layers": None, "recomputed_layers": None})
        return s

