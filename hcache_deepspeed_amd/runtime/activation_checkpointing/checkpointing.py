"""Activation checkpointing (reference: runtime/activation_checkpointing/checkpointing.py -- ``checkpoint`` :488,
``non_reentrant_checkpoint`` :704, ``configure``, model-parallel RNG tracker :124-247, cpu_checkpointing :474-486,
partition_activations :266-303 / :377-431, contiguous buffers, ``profile``).

Implementation: torch's non-reentrant checkpoint (saved-tensor hooks), which composes with the ZeRO-3 forward hooks
(a recomputed block re-gathers its unit) and with the host activation cache. ``cpu_checkpointing`` keeps the block
inputs in pinned host memory via ``torch.autograd.graph.save_on_cpu(pin_memory=True)``.

``partition_activations`` (tensor parallelism, where every model-parallel rank holds the same block inputs): each
rank keeps only its 1/mp slice of every floating checkpointed input (``_PartitionedCheckpoint``: the slices go
through ``save_for_backward``, so the host activation cache or ``cpu_checkpointing`` can move them too) and the
recompute all-gathers them over the model-parallel group first. ``contiguous_memory_optimization`` stores those
slices in ONE preallocated buffer per input position with ``number_checkpoints`` slots (no allocator churn between
layers; ``reset()`` rewinds it every forward), and requires ``number_checkpoints``. ``profile`` times every
checkpointed forward and recompute (synchronised) and logs the totals at ``reset()``.
"""
import contextlib
import functools
import time

import torch
import torch.utils.checkpoint as _tc

from ... import comm as dist

_CONFIG = {"partition_activations": False, "contiguous_memory_optimization": False, "cpu_checkpointing": False,
           "number_checkpoints": None, "synchronize_checkpoint_boundary": False, "profile": False}
_MPU = None
_CONFIGURED = False


def configure(mpu_, deepspeed_config=None, partition_activations=None, contiguous_checkpointing=None,
              num_checkpoints=None, checkpoint_in_cpu=None, synchronize=None, profile=None):
    global _MPU, _CONFIGURED
    _MPU = mpu_
    if deepspeed_config is not None:
        from ..config import DeepSpeedConfig
        cfg = deepspeed_config if isinstance(deepspeed_config, DeepSpeedConfig) else DeepSpeedConfig(
            deepspeed_config, world_size=1)
        ac = cfg.activation_checkpointing_config
        _CONFIG.update(partition_activations=ac.partition_activations,
                       contiguous_memory_optimization=ac.contiguous_memory_optimization,
                       cpu_checkpointing=ac.cpu_checkpointing, number_checkpoints=ac.number_checkpoints,
                       synchronize_checkpoint_boundary=ac.synchronize_checkpoint_boundary, profile=ac.profile)
    for k, v in (("partition_activations", partition_activations),
                 ("contiguous_memory_optimization", contiguous_checkpointing), ("number_checkpoints", num_checkpoints),
                 ("cpu_checkpointing", checkpoint_in_cpu), ("synchronize_checkpoint_boundary", synchronize),
                 ("profile", profile)):
        if v is not None:
            _CONFIG[k] = v
    if _CONFIG["contiguous_memory_optimization"] and not _CONFIG["number_checkpoints"]:
        raise ValueError("activation_checkpointing.contiguous_memory_optimization needs number_checkpoints (the slots "
                         "of its preallocated buffers)")
    _CONTIG.bufs.clear()
    _CONFIGURED = True


def is_configured():
    return _CONFIGURED


class _Contiguous:
    """One preallocated flat buffer per checkpointed-input position, ``number_checkpoints`` slots each."""

    def __init__(self):
        self.bufs = {}  # position -> (buffer [slots, n], next slot)

    def take(self, pos, part):
        slots = _CONFIG["number_checkpoints"]
        b = self.bufs.get(pos)
        if b is None or b[0].shape[1] != part.numel() or b[0].dtype != part.dtype or b[0].device != part.device:
            b = [torch.empty(slots, part.numel(), dtype=part.dtype, device=part.device), 0]
            self.bufs[pos] = b
        if b[1] >= slots:
            raise RuntimeError(f"contiguous_memory_optimization: more than number_checkpoints={slots} checkpointed "
                               f"calls since the last reset()")
        buf, i = b[0], b[1]
        b[1] += 1
        # a slot tensor over the buffer's storage WITHOUT the view relationship: views share one version counter,
        # so filling a later slot would invalidate the earlier slots saved for backward
        n = part.numel()
        out = torch.empty(0, dtype=part.dtype, device=part.device).set_(buf.untyped_storage(),
                                                                        buf.storage_offset() + i * n, (n, ))
        out.copy_(part)
        return out

    def rewind(self):
        for b in self.bufs.values():
            b[1] = 0


_CONTIG = _Contiguous()
_STATS = {"calls": 0, "saved_bytes": 0, "full_bytes": 0, "fwd_s": 0.0, "recompute_s": 0.0}


def stats():
    """Counters since the last ``reset()``: checkpointed calls, bytes of inputs kept (after partitioning) against
    their full size, and with ``profile`` the synchronised forward / recompute seconds."""
    return dict(_STATS)


def reset():
    """Start of a new forward (reference ``reset``): rewind the contiguous buffers, log and clear the profile."""
    if _CONFIG["profile"] and _STATS["calls"]:
        from ...utils.logging import log_dist
        log_dist(f"activation checkpointing: {_STATS['calls']} calls, forward {_STATS['fwd_s'] * 1e3:.1f} ms, "
                 f"recompute {_STATS['recompute_s'] * 1e3:.1f} ms, kept {_STATS['saved_bytes'] / 2**20:.1f} of "
                 f"{_STATS['full_bytes'] / 2**20:.1f} MiB", ranks=[0])
    _CONTIG.rewind()
    for k in _STATS:
        _STATS[k] = 0.0 if k.endswith("_s") else 0


def _mp_group():
    if _MPU is not None:
        g = _MPU.get_model_parallel_group() if hasattr(_MPU, "get_model_parallel_group") else None
    else:
        from ...utils import groups
        g = groups._get_model_parallel_group() if dist.is_initialized() else None
    if g is None or dist.get_world_size(g) <= 1:
        return None
    return g


def _partitionable(t, mp):
    return torch.is_tensor(t) and t.is_floating_point() and t.numel() >= mp


class _Timer:

    def __init__(self, key):
        self.key = key

    def __enter__(self):
        if _CONFIG["profile"]:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        if _CONFIG["profile"]:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            _STATS[self.key] += time.perf_counter() - self.t0


def _rng_snapshot():
    """Forward-time RNG states a recompute must replay: the CPU and device generators and the model-parallel tracker's
    named states (reference checkpointing.py:539,645-660 -- dropout inside model-parallel regions draws from the
    tracker, so without it the recomputed masks differ from the forward's and the gradients are silently wrong)."""
    dev = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
    return torch.get_rng_state(), dev, get_cuda_rng_tracker().get_states()


@contextlib.contextmanager
def _replay_rng(ctx):
    """Run the recompute under the forward's RNG states; afterwards restore the backward-time states (CPU, device and
    tracker) so the recompute consumes no randomness of the surrounding program."""
    devs = [torch.cuda.current_device()] if ctx.dev_rng is not None else []
    tracker = get_cuda_rng_tracker()
    bwd_tracker = tracker.get_states()
    with torch.random.fork_rng(devices=devs):
        torch.set_rng_state(ctx.cpu_rng)
        if ctx.dev_rng is not None:
            torch.cuda.set_rng_state(ctx.dev_rng)
        tracker.set_states(dict(ctx.tracker_rng))
        try:
            yield
        finally:
            tracker.set_states(bwd_tracker)


class _PartitionedCheckpoint(torch.autograd.Function):
    """Reentrant checkpoint that keeps 1/mp of each floating input (see module docstring)."""

    @staticmethod
    def forward(ctx, run, group, *args):
        mp, r = dist.get_world_size(group), dist.get_rank(group)
        ctx.run, ctx.group = run, group
        ctx.meta = []  # per arg: None (kept whole / non-tensor) or (shape, numel, requires_grad)
        keep, saved = [], []
        for i, a in enumerate(args):
            if _partitionable(a, mp):
                flat = a.detach().reshape(-1)
                part_n = -(-flat.numel() // mp)
                lo, hi = min(r * part_n, flat.numel()), min((r + 1) * part_n, flat.numel())
                part = flat.new_zeros(part_n)
                part[:hi - lo] = flat[lo:hi]
                if _CONFIG["contiguous_memory_optimization"]:
                    part = _CONTIG.take(len(saved), part)
                ctx.meta.append((a.shape, flat.numel(), a.requires_grad))
                saved.append(part)
                keep.append(None)
                _STATS["saved_bytes"] += part.numel() * part.element_size()
                _STATS["full_bytes"] += flat.numel() * flat.element_size()
            else:
                ctx.meta.append(None)
                keep.append(a)
        ctx.keep = keep
        ctx.save_for_backward(*saved)
        ctx.cpu_rng, ctx.dev_rng, ctx.tracker_rng = _rng_snapshot()
        _STATS["calls"] += 1
        with torch.no_grad(), _Timer("fwd_s"):
            out = run(*args)
        ctx.tuple_out = isinstance(out, tuple)
        return out

    @staticmethod
    def backward(ctx, *gouts):
        parts = list(ctx.saved_tensors)
        mp = dist.get_world_size(ctx.group)
        args = []
        for m, k in zip(ctx.meta, ctx.keep):
            if m is None:
                args.append(k)
                continue
            shape, n, rg = m
            part = parts.pop(0)
            full = part.new_empty(part.numel() * mp)
            dist.all_gather_into_tensor(full, part.contiguous(), group=ctx.group)
            args.append(full[:n].view(shape).requires_grad_(rg))
        with _replay_rng(ctx), _Timer("recompute_s"):
            with torch.enable_grad():
                out = ctx.run(*args)
        outs = out if ctx.tuple_out else (out, )
        pairs = [(o, g) for o, g in zip(outs, gouts) if torch.is_tensor(o) and o.requires_grad and g is not None]
        if pairs:
            torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        return (None, None) + tuple(a.grad if torch.is_tensor(a) and a.requires_grad else None for a in args)


def checkpoint(function, *args, **kwargs):
    """Recompute ``function(*args)`` in backward instead of storing its activations (with ``partition_activations``
    under tensor parallelism: keeping 1/mp of the inputs, all-gathered on recompute)."""
    ctx = contextlib.nullcontext()
    if _CONFIG["cpu_checkpointing"]:
        ctx = torch.autograd.graph.save_on_cpu(pin_memory=torch.cuda.is_available())
    if _CONFIG["synchronize_checkpoint_boundary"] and torch.cuda.is_available():
        torch.cuda.synchronize()
    group = _mp_group() if _CONFIG["partition_activations"] else None
    if group is not None and torch.is_grad_enabled():
        fn = functools.partial(function, **kwargs) if kwargs else function
        with ctx:
            return _PartitionedCheckpoint.apply(fn, group, *args)
    if _CONFIG["profile"] or _CONFIG["contiguous_memory_optimization"]:
        _STATS["calls"] += 1
        for a in args:
            if torch.is_tensor(a) and a.is_floating_point():
                nb = a.numel() * a.element_size()
                _STATS["saved_bytes"] += nb
                _STATS["full_bytes"] += nb
    if get_cuda_rng_tracker().get_states() and "context_fn" not in kwargs:
        kwargs["context_fn"] = _tracker_context_fn
    with ctx, _Timer("fwd_s"):
        return _tc.checkpoint(function, *args, use_reentrant=False, **kwargs)


def _tracker_context_fn():
    """torch non-reentrant checkpoint ``context_fn``: the forward snapshots the model-parallel RNG tracker, the
    recompute runs under that snapshot and restores the backward-time states after (torch itself replays only the
    CPU / device generators)."""
    snap = {}
    tracker = get_cuda_rng_tracker()

    @contextlib.contextmanager
    def fwd():
        snap["s"] = tracker.get_states()
        yield

    @contextlib.contextmanager
    def rec():
        bwd = tracker.get_states()
        tracker.set_states(dict(snap["s"]))
        try:
            yield
        finally:
            tracker.set_states(bwd)

    return fwd(), rec()


non_reentrant_checkpoint = checkpoint


class _SavedInputCheckpoint(torch.autograd.Function):
    """Checkpoint whose differentiable inputs go through ``ctx.save_for_backward`` -- and therefore through any
    enclosing ``saved_tensors_hooks``, e.g. the host activation cache, which can then spill them to host memory and
    prefetch them for the backward (torch's non-reentrant checkpoint keeps its inputs in a closure, invisible to
    such hooks). Reference: the reentrant ``CheckpointFunction`` with ``cpu_checkpointing``
    (runtime/activation_checkpointing/checkpointing.py:474-486), here asynchronous via the cache's copy stream."""

    @staticmethod
    def forward(ctx, run, stash_attention, *args):
        from ...ops.attention import AttnStash
        ctx.run = run
        ctx.grad_idx = [i for i, a in enumerate(args) if torch.is_tensor(a) and a.requires_grad]
        ctx.others = [None if i in ctx.grad_idx else a for i, a in enumerate(args)]
        ctx.cpu_rng, ctx.dev_rng, ctx.tracker_rng = _rng_snapshot()
        stash = []
        prev = (AttnStash.mode, AttnStash.items)
        if stash_attention:
            AttnStash.mode, AttnStash.items = "record", stash
        try:
            with torch.no_grad():
                out = run(*args)
        finally:
            AttnStash.mode, AttnStash.items = prev
        ctx.n_stash = len(stash)
        # the attention outputs go through save_for_backward next to the inputs: an enclosing host activation cache
        # spills them like the inputs (ckpt_offload), and the recompute replays them instead of re-running attention.
        # Made under no_grad they are autograd leaves, which the cache leaves alone (parameters are leaves too): the
        # mark says these are activations
        for pair in stash:
            for t in pair:
                t._hds_activation = True
        ctx.save_for_backward(*[args[i] for i in ctx.grad_idx], *[t for pair in stash for t in pair])
        ctx.tuple_out = isinstance(out, tuple)
        return out

    @staticmethod
    def backward(ctx, *gouts):
        from ...ops.attention import AttnStash
        saved = ctx.saved_tensors
        n_in = len(saved) - 2 * ctx.n_stash
        args = list(ctx.others)
        for i, t in zip(ctx.grad_idx, saved[:n_in]):
            args[i] = t.detach().requires_grad_(True)
        stash = [(saved[n_in + 2 * j], saved[n_in + 2 * j + 1]) for j in range(ctx.n_stash)]
        prev = (AttnStash.mode, AttnStash.items)
        if ctx.n_stash:
            AttnStash.mode, AttnStash.items = "replay", stash
        try:
            with _replay_rng(ctx):
                with torch.enable_grad():
                    out = ctx.run(*args)
        finally:
            AttnStash.mode, AttnStash.items = prev
        outs = out if ctx.tuple_out else (out, )
        pairs = [(o, g) for o, g in zip(outs, gouts) if torch.is_tensor(o) and o.requires_grad and g is not None]
        if pairs:
            torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        return (None, None) + tuple(args[i].grad if i in ctx.grad_idx else None for i in range(len(args)))


def checkpoint_saved_inputs(function, *args, stash_attention=False):
    """Recompute ``function(*args)`` in backward; its differentiable tensor inputs are saved through
    ``save_for_backward`` (host-cache visible, see ``_SavedInputCheckpoint``). Positional arguments only.
    ``stash_attention``: also keep every attention call's output + LSE (``ops.attention.AttnStash``) and replay them
    in the recompute, which then skips the FlashAttention forward -- at long context most of a block's recompute."""
    return _SavedInputCheckpoint.apply(function, bool(stash_attention), *args)


# ---------------------------------------------------------------------------------------------
# model-parallel RNG (reference :124-247): dropout masks identical across TP ranks for replicated
# regions and different for partitioned regions.
# ---------------------------------------------------------------------------------------------
_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"


class CudaRNGStatesTracker:

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = states

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception(f"seed {seed} already exists")
        self.seeds_.add(seed)
        if name in self.states_:
            raise Exception(f"cuda rng state {name} already exists")
        if not torch.cuda.is_available():
            self.states_[name] = torch.random.get_rng_state()
            return
        orig = torch.cuda.get_rng_state()
        torch.cuda.manual_seed(seed)
        self.states_[name] = torch.cuda.get_rng_state()
        torch.cuda.set_rng_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception(f"cuda rng state {name} is not added")
        cuda = torch.cuda.is_available()
        orig = torch.cuda.get_rng_state() if cuda else torch.random.get_rng_state()
        (torch.cuda.set_rng_state if cuda else torch.random.set_rng_state)(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = torch.cuda.get_rng_state() if cuda else torch.random.get_rng_state()
            (torch.cuda.set_rng_state if cuda else torch.random.set_rng_state)(orig)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


def model_parallel_cuda_manual_seed(seed):
    tp_rank = _MPU.get_model_parallel_rank() if _MPU is not None else 0
    offset = seed + 2718
    mp_seed = offset + tp_rank
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
    _CUDA_RNG_STATE_TRACKER.reset()
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, mp_seed)
