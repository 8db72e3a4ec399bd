"""Activation checkpointing (reference: runtime/activation_checkpointing/checkpointing.py -- ``checkpoint`` :488,
``non_reentrant_checkpoint`` :704, ``configure``, model-parallel RNG tracker :124-247, cpu_checkpointing :474-486).

Implementation: torch's non-reentrant checkpoint (saved-tensor hooks), which composes with the ZeRO-3
forward hooks (a recomputed block re-gathers its unit) and with the host activation cache. ``cpu_checkpointing``
keeps the block inputs in pinned host memory via ``torch.autograd.graph.save_on_cpu(pin_memory=True)``.
``partition_activations`` splits checkpointed inputs across the tensor-parallel group and all-gathers them
on recompute.
"""
import contextlib

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
    _CONFIGURED = True


def is_configured():
    return _CONFIGURED


def reset():
    pass


class _PartitionedInput(torch.autograd.Function):
    """Keep only this TP rank's slice of a checkpointed activation; all-gather it on recompute."""

    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        return g


def checkpoint(function, *args, **kwargs):
    """Recompute ``function(*args)`` in backward instead of storing its activations."""
    ctx = contextlib.nullcontext()
    if _CONFIG["cpu_checkpointing"]:
        ctx = torch.autograd.graph.save_on_cpu(pin_memory=torch.cuda.is_available())
    if _CONFIG["synchronize_checkpoint_boundary"] and torch.cuda.is_available():
        torch.cuda.synchronize()
    with ctx:
        return _tc.checkpoint(function, *args, use_reentrant=False, **kwargs)


non_reentrant_checkpoint = checkpoint


class _SavedInputCheckpoint(torch.autograd.Function):
    """Checkpoint whose differentiable inputs go through ``ctx.save_for_backward`` -- and therefore through any
    enclosing ``saved_tensors_hooks``, e.g. the host activation cache, which can then spill them to host memory and
    prefetch them for the backward (torch's non-reentrant checkpoint keeps its inputs in a closure, invisible to
    such hooks). Reference: the reentrant ``CheckpointFunction`` with ``cpu_checkpointing``
    (runtime/activation_checkpointing/checkpointing.py:474-486), here asynchronous via the cache's copy stream."""

    @staticmethod
    def forward(ctx, run, n_out_hint, *args):
        ctx.run = run
        ctx.grad_idx = [i for i, a in enumerate(args) if torch.is_tensor(a) and a.requires_grad]
        ctx.others = [None if i in ctx.grad_idx else a for i, a in enumerate(args)]
        ctx.save_for_backward(*[args[i] for i in ctx.grad_idx])
        ctx.cpu_rng = torch.get_rng_state()
        ctx.dev_rng = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        with torch.no_grad():
            out = run(*args)
        ctx.tuple_out = isinstance(out, tuple)
        return out

    @staticmethod
    def backward(ctx, *gouts):
        saved = ctx.saved_tensors
        args = list(ctx.others)
        for i, t in zip(ctx.grad_idx, saved):
            args[i] = t.detach().requires_grad_(True)
        devs = [torch.cuda.current_device()] if ctx.dev_rng is not None else []
        with torch.random.fork_rng(devices=devs):
            torch.set_rng_state(ctx.cpu_rng)
            if ctx.dev_rng is not None:
                torch.cuda.set_rng_state(ctx.dev_rng)
            with torch.enable_grad():
                out = ctx.run(*args)
        outs = out if ctx.tuple_out else (out, )
        pairs = [(o, g) for o, g in zip(outs, gouts) if torch.is_tensor(o) and o.requires_grad and g is not None]
        if pairs:
            torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        return (None, None) + tuple(args[i].grad if i in ctx.grad_idx else None for i in range(len(args)))


def checkpoint_saved_inputs(function, *args):
    """Recompute ``function(*args)`` in backward; its differentiable tensor inputs are saved through
    ``save_for_backward`` (host-cache visible, see ``_SavedInputCheckpoint``). Positional arguments only."""
    return _SavedInputCheckpoint.apply(function, 0, *args)


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
