"""Training-side host activation cache ("Hcache" for training): spill saved activations to pinned host DRAM.

BASELINE north star: "activations ... spill to host DRAM without stalling backward". Reference analogues:
CPU activation checkpointing (runtime/activation_checkpointing/checkpointing.py:59,474-486), FPDT chunk
offload (sequence/fpdt_layer.py:462-508 ``SequenceChunk``) and the DeepCompile offload_activation pass
(compile/passes/offload_activation.py, csrc/compile/z3.cpp:268-341).

Mechanism (``torch.autograd.graph.saved_tensors_hooks``):

* forward/pack: a saved activation larger than ``min_bytes`` from a block that is not among the last
  ``min_layers_resident`` blocks is copied D2H on a dedicated HIP copy stream into a pinned host buffer
  from a reuse pool (``offload/pinned.py``, hipHostMalloc). The GPU tensor is released immediately with
  ``record_stream`` so the caching allocator recycles it once the DMA has drained -- forward never waits.
* backward/unpack: when backward first touches ANY saved tensor of block i (spilled or resident -- resident
  tensors of tracked blocks carry a small layer tag for exactly this), the spilled tensors of blocks
  i-1 .. i-prefetch_layers are prefetched H2D on the copy stream (reverse layer order), so the PCIe transfer
  overlaps the backward of the blocks after them; the compute stream only waits on the per-tensor HIP event.
  (Tagging resident tensors matters under the budget policy: the spilled blocks are the EARLIEST ones, whose
  successors are all resident -- without the tag nothing would start their prefetch before they are needed.)
Parameters (autograd leaves) and small tensors are never offloaded.

Budget policy (``gpu_budget_bytes``): spilling everything is PCIe-bound (at 32k tokens a Llama-3-8B layer saves
~4.6 GB; 30 layers both ways is ~300 GB per step), so only what does not fit in HBM is spilled. The first
(calibration) step spills every eligible layer and records each layer's eligible bytes plus the step's peak
allocation; from then on only the *earliest* layers 0..k-1 are spilled, with k the smallest prefix that keeps
``peak_all + resident_bytes(k..)`` under the budget (``plan_offload``). Early layers are spilled because their
D2H has the whole remaining forward to drain and their H2D the whole remaining backward to prefetch. A runtime
guard still spills any tensor that would push the allocation past the budget.

``policy="ckpt_offload"`` checkpoints EVERY block (``checkpoint_saved_inputs``: its differentiable inputs are saved
through ``save_for_backward``, so the pack hook below sees them) and spills those inputs -- the residual stream, two
[tokens, hidden] tensors per block -- with no budget: the long-context mode, where even the checkpoints exceed HBM
(Llama-3-8B at 256k tokens: 4.3 GB per block, 137 GB for 32 blocks, against ~95 s of compute per step).

``policy="auto"`` (spill + recompute): starts as ``recompute``; after the first planned step it moves the EARLIEST
planned blocks to spilling, as many as the copy stream can drain inside a fraction ``spill_overlap`` of the forward:
k = spill_overlap * t_forward / (block bytes / PCIe rate), with the PCIe rate measured on the calibration step's
copies and t_forward on the first planned step. Those blocks then cost no recompute, the rest are recomputed.

``policy="recompute"`` plans the same over-budget layers but recomputes them in backward (non-reentrant activation
checkpointing of just those blocks) instead of spilling them: when PCIe cannot hide the spill (at 32k tokens a
Llama-3-8B layer moves ~3.5 GB each way, ~61 ms per direction against ~27 ms to recompute its forward), selective
recomputation is the cheaper way to meet the budget; the closed-loop refinement below applies to either set.

Two corrections keep the budgeted cache off the critical path:
* the calibration peak over-states the all-spilled peak (spilled tensors still waiting for their D2H hold HBM
  inside the copy window), so after each planned step the forward/backward turn-around peak is compared with the
  budget and the latest spilled layers whose bytes fit in the slack are kept resident from then on (closed loop);
* in backward the spilled layers are prefetched as far ahead as the HBM the backward has already freed allows
  (bounded by the budget), not only ``prefetch_layers`` ahead: the H2D of the spilled prefix then overlaps the
  backward of the resident layers instead of bunching up at the end of the step.
"""
import contextlib
import functools
import os
import sys
import time

import torch
import torch.nn as nn

from ..utils.logging import log_dist, logger
from ..ops.hostcopy import d2h_
from .pinned import PinnedPool


def default_host_budget_gib():
    """Pinned host bytes one rank's cache may hold: 40 % of the host's RAM (at most 160 GiB) shared by the ranks
    running on this node -- eight GPUs spill into one host's DRAM."""
    import psutil
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    return min(0.4 * psutil.virtual_memory().total / 2**30 / local, 160.0)


class _Spilled:
    __slots__ = ("host", "shape", "dtype", "device", "layer", "d2h_done", "dev", "h2d_done", "stride_ok")

    def __init__(self):
        self.dev = None
        self.h2d_done = None


class _Tagged:
    """A resident saved tensor of a tracked block: unpacking it tells the cache where backward is."""
    __slots__ = ("t", "layer")

    def __init__(self, t, layer):
        self.t, self.layer = t, layer


class HostActivationCache:

    def __init__(self, device, min_bytes=1 << 20, min_layers_resident=2, prefetch_layers=1,
                 gpu_budget_bytes=None, host_budget_bytes=None, copy_window_bytes=None, recompute=False,
                 ckpt_offload=False, hybrid=False, spill_overlap=0.5, stash_attention=True):
        self.device = device
        self.stash_attention = bool(stash_attention)  # ckpt_offload: keep attention outputs, skip FA in recompute
        self.hybrid = bool(hybrid)  # policy "auto": recompute plan, then the earliest blocks switch to spilling
        self.policy_recompute = bool(recompute) or self.hybrid
        self.ckpt_offload = bool(ckpt_offload)
        self.spill_overlap = float(spill_overlap)
        self._hybrid_state = 0  # 0: not planned, 1: first planned step running (timed), 2: split done
        self._fwd_ev = None  # (start, end) timing events of the last forward
        self._cal_copy = [None, None, 0]  # calibration copies: first-start event, last-end event, bytes
        self.pcie_gbps = None
        self.recompute = set()  # blocks whose forward is checkpointed (policy "recompute")
        self.resident_block_bytes = 0  # measured device footprint of a block kept resident (recompute policies)
        self._blk_mark = None
        # D2H copy window: spilled bytes the host may have queued on the copy stream and not yet seen copied.
        # Autograd runs far ahead of the GPU on the host, and a spilled tensor's HBM is recycled only once its D2H
        # drained (record_stream) -- with PCIe slower than a layer's forward the backlog grows layer by layer. Left
        # unbounded it exhausts the allocator, which then frees its cache behind a device-wide synchronize; the
        # window keeps it inside the HBM the budget leaves free (the host waits only when it would not fit). The
        # backward needs no window: prefetch buffers are allocated and consumed on the compute stream and the
        # copy stream waits for them (see _prefetch), so their blocks recycle in stream order.
        # Under an HBM budget the bytes in flight count AGAINST the budget: a spilled tensor's HBM returns only once its
        # D2H has drained. Round 4 sized the window from the HBM outside the budget (52 GiB at a 230 GiB budget on
        # 288 GiB), which let in-flight spills carry the step to 250 GiB. Now it is a small slice of the budget
        # (budget / 32, 64 MiB .. 4 GiB: at 230 GiB, 4 GiB = ~75 ms of PCIe backlog), and the plans, closed-looped on the
        # measured peaks, keep those bytes inside the budget.
        if copy_window_bytes is None:
            copy_window_bytes = 16 << 30
            if gpu_budget_bytes is not None and device.type == "cuda":
                copy_window_bytes = int(min(4 << 30, max(64 << 20, gpu_budget_bytes // 32)))
        self.copy_window = int(copy_window_bytes)
        self._d2h_q, self._h2d_q = [], []
        # host waits on the copy window: the HOST blocks until the oldest queued spill drained. The GPU keeps
        # running the kernels queued before it (autograd is ahead of the device), so this is host time, not a device
        # stall, as long as the queue ahead of the copy is not empty (throttle_wait_s: total host seconds waited)
        self.throttle_waits = 0
        self.throttle_wait_s = 0.0
        # pinned host bytes the cache may hold at once (the calibration step spills every eligible layer; at long
        # context that alone can exceed the host's memory): beyond it tensors stay on the GPU
        self.host_budget = host_budget_bytes
        self.host_in_use = 0
        self.budget = gpu_budget_bytes  # None: spill every eligible layer (no planning)
        self.plan = None  # set of layer indices to spill once calibrated
        self.layer_bytes = {}
        self._calibrating = False
        self.min_bytes = int(min_bytes)
        self.keep = int(min_layers_resident)
        self.prefetch_layers = int(prefetch_layers)
        self.pool = PinnedPool()
        # high priority: HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues round-robin, and a copy that
        # lands in the compute stream's queue cannot start before every kernel queued ahead of it has finished
        self.stream = torch.cuda.Stream(device, priority=-1) if device.type == "cuda" else None
        # backward prefetches get their own stream: on the D2H stream they queued behind the forward's spill backlog
        # (up to the copy window) and the first recomputed block of a 128k ckpt_offload step waited 191 ms for them
        self.h2d_stream = torch.cuda.Stream(device, priority=-1) if device.type == "cuda" else None
        self.cur_layer = -1
        self.n_layers = 0
        self.by_layer = {}
        self.bytes_offloaded = 0
        # diagnostics: saved tensors unpacked before their prefetch was issued (a compute-stream stall on PCIe),
        # tensors the runtime guard spilled outside the plan, bytes the host cap kept on the GPU
        self.late_unpacks = 0
        self.guard_spills = 0
        self.host_capped_bytes = 0
        self.stashed_blocks = 0  # ckpt_offload blocks whose attention output was stashed in the last forward
        self.stash_keep_from = 1 << 30  # blocks from here on keep their stash on the device (_update_stash_keep)
        self._stash_sb = 0
        self._steps_seen = 0
        self._capped_this_step = 0
        self._attached = []
        self._wrapped = []  # blocks whose forward attach() wrapped (restored by detach)
        self._cal_recompute = set()  # blocks checkpointed during the calibration step (pinned budget used up)
        self._last_layer_bytes = 0
        self._cal_bytes = {}  # per-layer eligible bytes measured by the calibration step
        self._turn_peak = None  # max allocation at the forward/backward turn-around of the last step
        self.plan_adjustments = 0
        self.peak_seen = 0  # max allocation over every step (the planner resets the peak counter per forward)
        # the allocator's peak counter is reset per forward AND per backward block (bwd_headroom); the running max of
        # the step across those resets is what every calibration must read, not the raw counter
        self._step_max = 0
        self.last_step_peak = 0  # full peak of the previous step (set at the next forward)
        self.step_peak_history = []  # every finished step's full peak, in order (bench.py: the timed steps' max)
        # how far a step's peak rose above its forward/backward turn-around peak (backward transients: recompute,
        # prefetched spills, gradients): the plans keep the turn-around peak under budget - bwd_extra, so the WHOLE
        # step stays under the budget (max over the steps seen: conservative)
        self.bwd_extra = 0
        self._bwd_extra_cal, self._bwd_extra_planned = 0, None
        self.bwd_headroom = None  # largest one-block backward transient seen (bytes), kept free by far prefetches
        self._bwd_layer, self._bwd_mark = None, None
        self.bwd_layer_seen = None

    @classmethod
    def from_config(cls, cfg, device):
        budget = None
        if getattr(cfg, "policy", "budget") in ("budget", "recompute", "auto") and device.type == "cuda":
            gib = float(getattr(cfg, "gpu_budget_gib", 0.0) or 0.0)
            total = torch.cuda.get_device_properties(device).total_memory
            budget = int(gib * 2**30) if gib > 0 else int(0.92 * total)
        hgib = float(getattr(cfg, "host_budget_gib", 0.0) or 0.0)
        if hgib <= 0:
            hgib = default_host_budget_gib()
        wgib = float(getattr(cfg, "copy_window_gib", 0.0) or 0.0)
        return cls(device, min_bytes=int(float(getattr(cfg, "min_kib", 1024)) * 1024),
                   min_layers_resident=cfg.min_layers_resident,
                   prefetch_layers=int(getattr(cfg, "prefetch_layers", 2)), gpu_budget_bytes=budget,
                   host_budget_bytes=int(hgib * 2**30), copy_window_bytes=int(wgib * 2**30) if wgib > 0 else None,
                   recompute=getattr(cfg, "policy", "budget") == "recompute",
                   ckpt_offload=getattr(cfg, "policy", "budget") == "ckpt_offload",
                   hybrid=getattr(cfg, "policy", "budget") == "auto",
                   spill_overlap=float(getattr(cfg, "spill_overlap", 0.5)),
                   stash_attention=bool(getattr(cfg, "stash_attention", True)))

    # ---------------------------------------------------------------------------------------
    def attach(self, model):
        """Track which transformer block is running (every nn.ModuleList element counts as a block)."""
        blocks = []
        for m in model.modules():
            if isinstance(m, nn.ModuleList):
                blocks.extend(list(m))
        self.n_layers = len(blocks)
        if self.ckpt_offload:
            # models that support it checkpoint the summed residual stream: one spilled tensor per block, not two
            for m in model.modules():
                if hasattr(m, "summed_boundary"):
                    m.summed_boundary = True
        for i, b in enumerate(blocks):
            self._attached.append(b.register_forward_pre_hook(lambda mod, args, i=i: self._enter(i)))
            if self.policy_recompute:
                self._attached.append(b.register_forward_hook(lambda mod, args, out, i=i: self._exit(i, out)))
                b.forward = self._recompute_wrapper(b.forward, i)
                self._wrapped.append(b)
            elif self.ckpt_offload:
                b.forward = self._ckpt_offload_wrapper(b.forward)
                self._wrapped.append(b)
        return self

    def detach(self):
        """Undo ``attach`` (engine.destroy()): remove the block hooks, restore the blocks' own forwards, drop the
        pinned pool's buffers."""
        for h in self._attached:
            h.remove()
        self._attached = []
        for b in self._wrapped:
            b.__dict__.pop("forward", None)
        self._wrapped = []
        pool = getattr(self, "pool", None)
        if pool is not None and hasattr(pool, "clear"):
            pool.clear()

    def _ckpt_offload_wrapper(self, fwd):
        from ..runtime.activation_checkpointing import checkpointing as ck
        stash = self.stash_attention

        def run(*args, **kwargs):
            if not torch.is_grad_enabled():
                return fwd(*args, **kwargs)
            if any(torch.is_tensor(v) and v.requires_grad for v in kwargs.values()):
                return ck.checkpoint(fwd, *args, **kwargs)  # still recomputed; such inputs stay on the device
            # the attention output + LSE are saved (and spilled) too: the recompute replays them and skips the
            # FlashAttention forward -- at 128k tokens most of a block's recompute for ~1/3 more spilled bytes. Only
            # while the pinned-host budget still holds this stash AND the inputs of every block after it: a stash the
            # host cap keeps on the device would cost HBM that the longest contexts do not have
            st = stash and self._stash_fits(args)
            self.stashed_blocks += int(st)
            if kwargs:
                return ck.checkpoint_saved_inputs(functools.partial(fwd, **kwargs), *args, stash_attention=st)
            return ck.checkpoint_saved_inputs(fwd, *args, stash_attention=st)

        return run

    def _stash_fits(self, args):
        hidden = next((a.numel() * a.element_size() for a in args if torch.is_tensor(a)), 0)
        self._stash_sb = int(1.02 * hidden)  # o (hidden-sized) + LSE
        if self.cur_layer >= self.stash_keep_from:
            return True  # this block's stash stays on the device (_update_stash_keep)
        if self.host_budget is None:
            return True
        inputs = sum(a.numel() * a.element_size() for a in args if torch.is_tensor(a))
        rest = max(0, self.n_layers - max(self.cur_layer, 0) - self.keep) * inputs  # later blocks' spilled inputs
        return self.host_in_use + rest + int(1.02 * hidden) <= self.host_budget  # o (hidden-sized) + LSE

    def _update_stash_keep(self):
        """ckpt_offload with the attention stash: the stash goes to host memory like the inputs (needed at 320k
        tokens), but where the HBM holds it, keeping it on the device saves its round trip over PCIe (128k: ~8 %).
        From the second step on, the HBM the previous step left free (85 % of the device minus the peak allocation;
        the margin covers the caching allocator's fragmentation, which at 128k tokens reserves ~80 GiB more than the
        peak allocation -- reusable, so the reserved peak would understate the room) keeps the stash of the last
        blocks on the device; it only grows."""
        self._steps_seen += 1
        if not (self.ckpt_offload and self.stash_attention and self.device.type == "cuda" and self._stash_sb
                and self._steps_seen >= 2):
            return
        total = torch.cuda.get_device_properties(self.device).total_memory
        room = int(0.85 * total) - self.last_step_peak  # the previous step's full peak (read before the reset)
        if room > self._stash_sb:
            keep_from = max(0, min(self.stash_keep_from, self.n_layers) - room // self._stash_sb)
            if keep_from != self.stash_keep_from:
                log_dist(f"host activation cache: attention stash of blocks {keep_from}..{self.n_layers - 1} stays "
                         f"on the device ({room / 2**30:.1f} GiB of HBM free at the peak)", ranks=[0])
                self.stash_keep_from = keep_from

    def _recompute_wrapper(self, fwd, i):
        from ..runtime.activation_checkpointing import checkpointing as ck

        def run(*args, **kwargs):
            if (i in self.recompute or i in self._cal_recompute) and torch.is_grad_enabled():
                return ck.checkpoint(fwd, *args, **kwargs)
            return fwd(*args, **kwargs)

        return run

    def _enter(self, i):
        if torch.is_grad_enabled():
            self.cur_layer = i
            # calibration of the recompute policies spills every eligible tensor; once the pinned-host budget is
            # nearly used up the remaining blocks of that step are checkpointed instead -- kept on the device their
            # activations would overflow the HBM (32k x mb2: ~290 GB of saved activations against a 160 GiB host
            # budget). Their per-layer bytes are filled in from the measured blocks when the plan is made.
            if (self._calibrating and self.policy_recompute and self.host_budget is not None
                    and i < self.n_layers - self.keep
                    and self.host_in_use + self._last_layer_bytes >= self.host_budget):
                self._cal_recompute.add(i)
            if self.policy_recompute and self.device.type == "cuda":
                self._blk_mark = (i, torch.cuda.memory_allocated(self.device))

    def _exit(self, i, out):
        """End of a block's forward (recompute policies): what a block kept on the device -- the growth of the
        allocation over its forward minus its output (which a checkpointed block holds too) -- measured on the blocks
        that were NOT checkpointed. The recompute plans price a block they stop recomputing with it: the bytes
        ``_pack`` counts miss what a block keeps outside the saved-tensor hooks, and at 32k x mb2 a plan sized from
        those counts kept 16 blocks resident and ran out of HBM in the next forward."""
        mark = getattr(self, "_blk_mark", None)
        self._blk_mark = None
        if mark is None or mark[0] != i or not torch.is_grad_enabled() or self.device.type != "cuda":
            return
        if i in self.recompute or i in self._cal_recompute or (self.plan and i in self.plan):
            return
        if self._calibrating and i < self.n_layers - self.keep:
            return  # spilled during calibration: its saved tensors left for the host
        outs = out if isinstance(out, (tuple, list)) else (out, )
        ob = sum(o.numel() * o.element_size() for o in outs if torch.is_tensor(o))
        kept = torch.cuda.memory_allocated(self.device) - mark[1] - ob
        self.resident_block_bytes = max(self.resident_block_bytes, kept)

    def _rc_bytes(self):
        """Per-block bytes the recompute plans use: the counted saved bytes, raised to the measured footprint of a
        resident block (``_exit``)."""
        rb = self.resident_block_bytes
        return {li: max(b, rb) for li, b in self._cal_bytes.items()}

    def _peak_fold(self):
        """The allocator's peak since its last reset, folded into the running max of this step."""
        pk = torch.cuda.max_memory_allocated(self.device)
        self._step_max = max(self._step_max, pk)
        return pk

    def _peak_reset(self):
        self._peak_fold()
        torch.cuda.reset_peak_memory_stats(self.device)

    def step_peak(self):
        """Peak allocation of the step running now (since its forward began), across the per-block resets."""
        if self.device.type != "cuda":
            return 0
        return max(self._step_max, torch.cuda.max_memory_allocated(self.device))

    def _take_step_peak(self):
        """Start of a forward: the whole previous step's peak (every reset inside it included) -> ``last_step_peak``,
        and a fresh running max for the step that starts now."""
        if self.device.type == "cuda":
            self.last_step_peak = max(self._step_max, torch.cuda.max_memory_allocated(self.device))
            self.peak_seen = max(self.peak_seen, self.last_step_peak)
            self.step_peak_history.append(self.last_step_peak)
            if self._turn_peak is not None:
                # the calibration step (everything spilled, prefetched back in backward) gives a conservative first
                # value; from the first planned step on, the max over the planned steps replaces it
                extra = max(0, self.last_step_peak - self._turn_peak)
                if self._was_calibrating():
                    self._bwd_extra_cal = extra
                else:
                    self._bwd_extra_planned = max(self._bwd_extra_planned or 0, extra)
                self.bwd_extra = (self._bwd_extra_planned if self._bwd_extra_planned is not None else
                                  self._bwd_extra_cal)
        self._step_max = 0
        return self.last_step_peak

    def _was_calibrating(self):
        """The step that just ended spilled every eligible tensor to measure (not a planned step)."""
        return bool(self._calibrating)

    def plan_budget(self):
        """The budget the forward-side plans aim the turn-around peak at (see ``bwd_extra``). Until a planned step has
        measured its own backward excess, the first plan also keeps the D2H copy window free: the calibration step
        it is sized from ran with nothing in that window at the turn-around, and the first planned 32k x mb2 step
        peaked 2.9 GiB over the budget without it (profiles/r5/plan_32768_mb2_r5full.json, ``step_peaks_gib``)."""
        if self.budget is None:
            return None
        first = self._bwd_extra_planned is None
        return self.budget - self.bwd_extra - (self.copy_window if first else 0)

    @contextlib.contextmanager
    def forward_context(self):
        if self.device.type == "cuda":
            self._take_step_peak()
        if self.budget is not None and self.device.type == "cuda":
            if self._calibrating:  # the previous step spilled everything: plan from what it measured
                # tensors the host cap kept on the GPU were all alive at the forward/backward turn-around, so the
                # "everything spilled" peak is the measured one minus them (plan_offload adds kept layers back)
                peak = self.last_step_peak - self._capped_this_step
                if self._cal_recompute:
                    # blocks the calibration checkpointed (host budget used up) saved only their inputs: plan them
                    # with the bytes the fully measured blocks saved (transformer blocks are alike)
                    full = [b for li, b in self.layer_bytes.items() if li not in self._cal_recompute]
                    if full:
                        mean = sum(full) // len(full)
                        for li in self._cal_recompute:
                            self.layer_bytes[li] = max(self.layer_bytes.get(li, 0), mean)
                    self._cal_recompute = set()
                self._cal_bytes = dict(self.layer_bytes)
                lb = self._rc_bytes() if self.policy_recompute else self.layer_bytes
                self.plan = calibrated_plan(lb, peak + self._capped_this_step, self._capped_this_step,
                                            self.plan_budget())
                self._calibrating = False
                if self.policy_recompute:  # the same over-budget layers, recomputed instead of spilled
                    self.recompute, self.plan = set(self.plan), set()
                    if self.hybrid:
                        self._hybrid_state = 1
                        self._measure_pcie()
                log_dist(f"host activation cache: spilling {len(self.plan)} of {self.n_layers} layers (peak when spilling all {peak / 2**30:.1f} GiB, budget "
                         f"{self.budget / 2**30:.1f} GiB, {self._capped_this_step / 2**30:.1f} GiB kept by the host cap)",
                         ranks=[0])
            elif self.plan is None:
                self._calibrating = True
            elif self.hybrid and self._hybrid_state == 1 and self._fwd_ev is not None:
                self._hybrid_split()
            elif self._turn_peak is not None:
                cur = self.recompute if self.policy_recompute else self.plan
                new = refine_plan(cur, self._rc_bytes() if self.policy_recompute else self._cal_bytes,
                                  self._turn_peak, self.plan_budget())
                if new != cur:
                    self.plan_adjustments += 1
                    if self.policy_recompute:
                        self.recompute = new
                    else:
                        self.plan = new
                    log_dist(f"host activation cache: turn-around peak {self._turn_peak / 2**30:.1f} GiB of "
                             f"{self.budget / 2**30:.1f} GiB -> {'recomputing' if self.policy_recompute else 'spilling'} "
                             f"{len(new)} layers", ranks=[0])
            self._turn_peak = None
        if self.device.type == "cuda":
            torch.cuda.reset_peak_memory_stats(self.device)
        self.cur_layer = -1
        for lst in self.by_layer.values():  # a forward whose backward never ran: return its host buffers
            for o in lst:
                if o.dev is not None and o.h2d_done is not None:
                    # a prefetch nobody consumed: its device buffer belongs to the compute stream's pool, and the
                    # H2D copy may still be writing it -- the compute stream must not reuse the block before then
                    torch.cuda.current_stream().wait_event(o.h2d_done)
                    o.dev = None
                if o.host is not None:
                    if o.h2d_done is not None and self.stream is not None:
                        # a prefetch nobody consumed may still read the buffer on the H2D stream: the next D2H into
                        # it (D2H stream) must come after it (consumed prefetches are ordered through the compute
                        # stream, which waited for them)
                        self.stream.wait_event(o.h2d_done)
                    self.host_in_use -= PinnedPool.nbytes_of(o.host)
                    self.pool.put(o.host)
                    o.host = None
        self.by_layer = {}
        self.layer_bytes = {}
        self._capped_this_step = 0
        self.stashed_blocks = 0
        self._bwd_layer, self._bwd_mark = None, None
        self.bwd_layer_seen = None
        self.bwd_events = []
        self._update_stash_keep()
        timed = self.hybrid and self._hybrid_state == 1 and self.device.type == "cuda"
        if timed:
            self._fwd_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self._fwd_ev[0].record()
        with torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack):
            yield
        if timed:
            self._fwd_ev[1].record()
        if self.device.type == "cuda" and self._turn_peak is None:
            # end of the forward: every saved activation is alive -- the turn-around peak the plan refinement uses
            self._turn_peak = torch.cuda.max_memory_allocated(self.device)

    def _measure_pcie(self):
        t0, t1, nbytes = self._cal_copy
        if t0 is not None and t1 is not None and nbytes > 0:
            t1.synchronize()
            ms = t0.elapsed_time(t1)
            if ms > 0:
                self.pcie_gbps = nbytes / ms / 1e6
        self._cal_copy = [None, None, 0]

    def _hybrid_split(self):
        """Policy "auto": move the earliest recomputed blocks to spilling -- as many as the copy stream drains within
        ``spill_overlap`` of the measured forward time (see module docstring)."""
        self._hybrid_state = 2
        s, e = self._fwd_ev
        e.synchronize()
        t_fwd_s = s.elapsed_time(e) / 1e3
        self._fwd_ev = None
        rec = sorted(self.recompute)
        if not rec or not self.pcie_gbps:
            return
        per = sum(self._cal_bytes.get(i, 0) for i in rec) / len(rec)
        t_copy = per / (self.pcie_gbps * 1e9)
        k = min(len(rec), int(self.spill_overlap * t_fwd_s / max(t_copy, 1e-9)))
        self.plan = set(rec[:k])
        self.recompute = set(rec[k:])
        log_dist(f"host activation cache (auto): forward {t_fwd_s * 1e3:.0f} ms, PCIe {self.pcie_gbps:.1f} GB/s, "
                 f"{per / 2**30:.2f} GiB per block -> spilling {k} and recomputing {len(rec) - k} of {len(rec)} "
                 f"over-budget blocks", ranks=[0])

    # ---------------------------------------------------------------------------------------
    def _window(self, q, nbytes):
        """Block the host until the copies queued in ``q`` leave room for ``nbytes`` more in the copy window."""
        while q and q[0][0].query():
            q.pop(0)
        while q and sum(b for _, b in q) + nbytes > self.copy_window:
            ev, _ = q.pop(0)
            t0 = time.perf_counter()
            ev.synchronize()
            self.throttle_wait_s += time.perf_counter() - t0
            self.throttle_waits += 1

    def _pack(self, t):
        if (not isinstance(t, torch.Tensor) or not t.is_cuda or self.cur_layer < 0
                or (t.is_leaf and not getattr(t, "_hds_activation", False))  # parameters, inputs; not the stash
                or t.numel() * t.element_size() < self.min_bytes):
            return t
        if getattr(t, "_hds_activation", False) and self.cur_layer >= self.stash_keep_from:
            return _Tagged(t, self.cur_layer) if self.by_layer else t  # a stash the HBM holds
        if self.cur_layer >= self.n_layers - self.keep:
            # kept resident, but tagged once something was spilled: backward touching these last blocks is what
            # starts the prefetch of the latest spilled ones
            return _Tagged(t, self.cur_layer) if self.by_layer else t
        nbytes = t.numel() * t.element_size()
        self.layer_bytes[self.cur_layer] = self.layer_bytes.get(self.cur_layer, 0) + nbytes
        self._last_layer_bytes = max(self._last_layer_bytes, self.layer_bytes[self.cur_layer])
        if self.plan is not None and self.cur_layer not in self.plan:
            if torch.cuda.memory_allocated(self.device) + nbytes <= self.budget:
                return _Tagged(t, self.cur_layer) if self.by_layer else t  # tag only when something was spilled
            self.guard_spills += 1
        if self.host_budget is not None and self.host_in_use + nbytes > self.host_budget:
            self.host_capped_bytes += nbytes
            self._capped_this_step += nbytes
            return _Tagged(t, self.cur_layer) if self.by_layer else t
        s = _Spilled()
        s.shape, s.dtype, s.device, s.layer = t.shape, t.dtype, t.device, self.cur_layer
        self._window(self._d2h_q, nbytes)
        src = t if t.is_contiguous() else t.contiguous()
        s.host = self.pool.get(src.numel(), src.dtype)
        ev = torch.cuda.Event()
        ev.record()
        cal = self.hybrid and self._calibrating
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            if cal and self._cal_copy[0] is None:  # PCIe rate of the calibration step's (saturating) copies
                self._cal_copy[0] = torch.cuda.Event(enable_timing=True)
                self._cal_copy[0].record(self.stream)
            d2h_(s.host, src.view(-1))  # few-workgroup copy kernel, not the wide blit (ops/hostcopy.py)
            src.record_stream(self.stream)
            s.d2h_done = torch.cuda.Event()
            s.d2h_done.record(self.stream)
            if cal:
                self._cal_copy[1] = torch.cuda.Event(enable_timing=True)
                self._cal_copy[1].record(self.stream)
                self._cal_copy[2] += nbytes
        self._d2h_q.append((s.d2h_done, nbytes))
        self.bytes_offloaded += src.numel() * src.element_size()
        self.host_in_use += PinnedPool.nbytes_of(s.host)  # the pinned bucket, not just the tensor
        self.by_layer.setdefault(s.layer, []).append(s)
        return s

    def _prefetch(self, s):
        if s.dev is not None or s.host is None:  # already fetched, or already consumed (host buffer returned)
            return
        # Allocate on the COMPUTE stream: its caching-allocator pool holds the blocks backward just freed, while
        # an allocation on the copy stream finds an empty per-stream pool and, with HBM nearly full, makes the
        # allocator free cached blocks -- a device-wide synchronize that serialises every copy with compute.
        cur = torch.cuda.current_stream()
        s.dev = torch.empty(s.shape, dtype=s.dtype, device=s.device)
        ready = torch.cuda.Event()
        ready.record(cur)
        with torch.cuda.stream(self.h2d_stream):
            self.h2d_stream.wait_event(s.d2h_done)  # the host copy must be complete
            self.h2d_stream.wait_event(ready)
            s.dev.view(-1).copy_(s.host, non_blocking=True)
            # no record_stream: the buffer was allocated on the compute stream after everything that used its block
            # (`ready`), and every later user of the block is a compute-stream kernel ordered after the consumer,
            # which waits for h2d_done -- so the block may recycle as soon as the consumer is enqueued
            s.h2d_done = torch.cuda.Event()
            s.h2d_done.record(self.h2d_stream)

    _DEBUG = os.environ.get("HDS_ACT_CACHE_DEBUG") == "1"

    track_progress = False  # bench.py heartbeat: one event per backward block, to report the GPU's position

    def _prefetch_before(self, layer):
        if layer != self.bwd_layer_seen:
            self.bwd_layer_seen = layer  # progress marker (host side: autograd runs ahead of the GPU)
            if self.track_progress and self.device.type == "cuda":
                ev = torch.cuda.Event()
                ev.record()
                self.bwd_events = (getattr(self, "bwd_events", []) + [(layer, ev)])[-64:]
        if self._turn_peak is None and self.device.type == "cuda":
            self._turn_peak = torch.cuda.max_memory_allocated(self.device)  # first unpack of the step
        if self.budget is not None and self.device.type == "cuda" and layer != self._bwd_layer:
            # backward reached a new block: the peak since the previous block began, over what was allocated then,
            # is what one block's backward (recompute intermediates + gradients) needs on top of the live tensors
            now = torch.cuda.memory_allocated(self.device)
            if self._bwd_mark is not None:
                pk = self._peak_fold()
                self.bwd_headroom = max(self.bwd_headroom or 0, pk - self._bwd_mark)
                self._peak_reset()
            self._bwd_layer, self._bwd_mark = layer, now
        # j = 0 first: the rest of THIS block's spilled tensors (a block unpacks several; if the first was late, the
        # others must not queue behind the earlier blocks' prefetches -- a 189 ms stall at 128k ckpt_offload)
        for j in range(0, self.prefetch_layers + 1):
            lst = self.by_layer.get(layer - j, ())
            if self._DEBUG and lst and lst[0].dev is None:
                print(f"[act-cache] t={time.perf_counter():.3f} backward at layer {layer}: prefetch layer {layer - j} "
                      f"({len(lst)} tensors), allocated {torch.cuda.memory_allocated(self.device) / 2**30:.1f} GiB",
                      file=sys.stderr, flush=True)
            for o in lst:
                self._prefetch(o)
        if self.budget is not None and self.device.type == "cuda":
            # further ahead, while the HBM the backward has already freed covers the next spilled layer AND leaves
            # one block's backward transient free (measured; a quarter of the budget until it has been): at 320k
            # tokens a block's recompute needs ~60 GB that greedy prefetching would otherwise have taken
            head = self.bwd_headroom if self.bwd_headroom is not None else self.budget // 4
            for lj in sorted((k for k in self.by_layer if k < layer - self.prefetch_layers), reverse=True):
                need = sum(o.host.numel() * o.host.element_size() for o in self.by_layer[lj]
                           if o.dev is None and o.host is not None)
                if need == 0:
                    continue
                if torch.cuda.memory_allocated(self.device) + need + head > self.budget:
                    break
                for o in self.by_layer[lj]:
                    self._prefetch(o)

    def _unpack(self, s):
        if isinstance(s, _Tagged):
            self._prefetch_before(s.layer)
            return s.t
        if not isinstance(s, _Spilled):
            return s
        if s.dev is None:
            self.late_unpacks += 1
        if self._DEBUG and s.dev is None:
            print(f"[act-cache] t={time.perf_counter():.3f} layer {s.layer} needed before its prefetch", file=sys.stderr,
                  flush=True)
        self._prefetch(s)
        self._prefetch_before(s.layer)
        torch.cuda.current_stream().wait_event(s.h2d_done)
        out = s.dev
        s.dev = None
        self.host_in_use -= PinnedPool.nbytes_of(s.host)
        self.pool.put(s.host)
        s.host = None
        return out

    def stats(self):
        return {"bytes_offloaded": self.bytes_offloaded, "pinned_pool_bytes": self.pool.bytes_allocated,
                "spilled_layers": None if self.plan is None else len(self.plan),
                "recomputed_layers": self.n_layers if self.ckpt_offload else len(self.recompute),
                "pcie_gbps": None if self.pcie_gbps is None else round(self.pcie_gbps, 1),
                "late_unpacks": self.late_unpacks,
                "guard_spills": self.guard_spills, "host_capped_bytes": self.host_capped_bytes,
                "stashed_blocks": self.stashed_blocks,
                "stash_on_device_blocks": max(0, self.n_layers - self.stash_keep_from) if self.ckpt_offload else 0,
                "bwd_headroom_gib": None if self.bwd_headroom is None else round(self.bwd_headroom / 2**30, 1),
                "copy_window_gib": round(self.copy_window / 2**30, 1), "throttle_waits": self.throttle_waits,
                "throttle_wait_s": round(self.throttle_wait_s, 2),
                "peak_gib_all_steps": round(self.peak_seen / 2**30, 1),
                "last_step_peak_gib": round(self.last_step_peak / 2**30, 2),
                "step_peaks_gib": [round(x / 2**30, 1) for x in self.step_peak_history[-16:]],
                "bwd_extra_gib": round(self.bwd_extra / 2**30, 2),
                "resident_block_gib": round(self.resident_block_bytes / 2**30, 2)}


def refine_plan(plan, layer_bytes, turn_peak, budget, margin=1 << 30):
    """Closed-loop correction of a spill plan (a prefix {0..k-1}) from the turn-around peak of a step that ran it:
    the latest spilled layers whose bytes fit in ``budget - margin - turn_peak`` stay resident from now on; a peak
    over the budget spills the following layers whose bytes cover the excess."""
    spilled = sorted(plan)
    slack = budget - margin - turn_peak
    if slack < 0:  # over budget: add the following layers until their bytes cover the excess (one step, not one
        # layer per step -- a plan refined from a low all-offloaded peak would otherwise creep back over many steps)
        nxt = (spilled[-1] + 1) if spilled else min(layer_bytes, default=None)
        need = -slack
        while need > 0 and nxt is not None and nxt in layer_bytes:
            spilled.append(nxt)
            need -= layer_bytes[nxt]
            nxt += 1
        return set(spilled)
    while spilled and layer_bytes.get(spilled[-1], 0) <= slack:
        slack -= layer_bytes.get(spilled[-1], 0)
        spilled.pop()
    return set(spilled)


def calibrated_plan(layer_bytes, measured_peak, host_capped_bytes, budget):
    """Plan from a calibration step in which the pinned-host cap kept ``host_capped_bytes`` of eligible tensors on
    the GPU: those bytes sit inside ``measured_peak`` (they are alive at the forward/backward turn-around) and are
    also counted in ``layer_bytes``, so the all-spilled peak is the measured one minus them."""
    return plan_offload(layer_bytes, measured_peak - host_capped_bytes, budget)


def plan_offload(layer_bytes, peak_all, budget):
    """Smallest prefix of layers to spill so the step peak stays under ``budget``.

    ``layer_bytes``: {layer: eligible saved bytes} measured while spilling all of them; ``peak_all``: the step's
    peak allocation in that state. Keeping layers k.. resident raises the peak by at most their bytes (they are
    all alive at the forward/backward turn-around). Returns the set {0..k-1}.
    """
    layers = sorted(layer_bytes)
    resident = 0
    k = len(layers)
    for i in reversed(range(len(layers))):
        if peak_all + resident + layer_bytes[layers[i]] > budget:
            break
        resident += layer_bytes[layers[i]]
        k = i
    return set(layers[:k])


class BlitLimitError(RuntimeError):
    """The host activation cache would spill through unlimited runtime blit kernels (see ``check_blit_limit``)."""


def check_blit_limit(cfg, device_type, limit_in_effect=None):
    """Warn -- or, in strict mode, refuse -- a spilling host activation cache when DEBUG_CLR_LIMIT_BLIT_WG did not
    reach the HIP runtime.

    Spills are device->host copies, which this ROCm stack runs as blit kernels spread over as many workgroups as the
    copy has chunks: they take CUs from the forward they overlap (32k tokens, 25 GiB spilled: 10,309 instead of
    13,949 tok/s, profiles/r4/copy_engine_ab_r4f.txt). The runtime reads the workgroup limit once, when it loads --
    i.e. at ``import torch`` -- so a script that imported torch before this package, without the variable exported,
    loses ~25 % of the overlapped forward. By default that is a loud warning with the fix (the run still trains
    correctly, only slower); ``host_act_cache.strict_blit_limit`` (or HDS_STRICT_BLIT=1) makes it a
    ``BlitLimitError`` at engine init. Policy "recompute" spills nothing; ``allow_unlimited_blit`` (or
    HDS_ALLOW_UNLIMITED_BLIT=1) silences both."""
    if device_type != "cuda":
        return
    if limit_in_effect is None:
        from .. import BLIT_LIMIT_EARLY as limit_in_effect
    if limit_in_effect or getattr(cfg, "policy", "budget") == "recompute":
        return
    if getattr(cfg, "allow_unlimited_blit", False) or os.environ.get("HDS_ALLOW_UNLIMITED_BLIT") == "1":
        logger.info("host activation cache: spills run as unlimited blit kernels (DEBUG_CLR_LIMIT_BLIT_WG was not "
                    "in the environment when torch loaded the HIP runtime); accepted by allow_unlimited_blit")
        return
    msg = ("host activation cache: DEBUG_CLR_LIMIT_BLIT_WG was not in the environment when torch loaded the HIP "
           "runtime, so activation spills run as unlimited blit kernels and slow the overlapped forward by ~25 %. Export "
           "DEBUG_CLR_LIMIT_BLIT_WG=16 before starting Python (the hcache_deepspeed_amd launcher and bench.py do), or "
           "import hcache_deepspeed_amd before torch; mi355x.host_act_cache.allow_unlimited_blit=true accepts it.")
    if getattr(cfg, "strict_blit_limit", False) or os.environ.get("HDS_STRICT_BLIT") == "1":
        raise BlitLimitError(msg)
    logger.warning(msg)


def build_activation_cache(cfg, device):
    """The cache for ``mi355x.host_act_cache`` (``cfg``): policy "plan" is the per-tensor planner
    (offload/act_plan.py), every other policy the block-level cache above."""
    check_blit_limit(cfg, device.type)
    if getattr(cfg, "policy", "budget") == "plan":
        from .act_plan import PlannedActivationCache
        return PlannedActivationCache.from_config(cfg, device)
    return HostActivationCache.from_config(cfg, device)
