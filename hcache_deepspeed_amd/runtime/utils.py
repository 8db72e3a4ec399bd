"""Runtime helpers (reference runtime/utils.py: ``clip_grad_norm_`` / ``get_global_norm`` with model-parallel
awareness, ``see_memory_usage``, ``get_grad_norm``, ``all_gather_dp_groups``, ``CheckOverflow``,
``partition_uniform``/``partition_balanced``, ``call_to_str``, ``graph_process`` capture helper)."""
import gc
import math

import psutil
import torch

from .. import comm as dist
from ..utils import groups
from ..utils.logging import logger
from .pipe.module import partition_balanced, partition_uniform  # noqa: F401  (re-export)


def _mp_group():
    return groups._get_model_parallel_group() if groups._State.topo is not None and \
        groups.get_model_parallel_world_size() > 1 else None


def get_global_norm(norm_list):
    return math.sqrt(sum(n**2 for n in norm_list))


def get_grad_norm(parameters, norm_type=2, mpu=None):
    """Global grad norm over data/model parallel ranks (tensor-parallel-replicated params counted once)."""
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return 0.0
    dev = params[0].grad.device
    if norm_type == float("inf"):
        tot = torch.stack([p.grad.detach().abs().max().float() for p in params]).max()
        g = _mp_group()
        if g is not None:
            dist.all_reduce(tot, op=dist.ReduceOp.MAX, group=g)
        return float(tot)
    sharded = torch.zeros((), device=dev)
    repl = torch.zeros((), device=dev)
    for p in params:
        v = p.grad.detach().float().norm(norm_type)**norm_type
        if getattr(p, "ds_tensor_model_parallel", False):
            sharded += v
        else:
            repl += v
    g = _mp_group()
    if g is not None:
        dist.all_reduce(sharded, group=g)
    return float((sharded + repl)**(1.0 / norm_type))


def clip_grad_norm_(parameters, max_norm, norm_type=2, mpu=None):
    parameters = list(parameters) if not isinstance(parameters, torch.Tensor) else [parameters]
    total = get_grad_norm(parameters, norm_type, mpu)
    coef = max_norm / (total + 1e-6)
    if coef < 1:
        for p in parameters:
            if p.grad is not None:
                p.grad.detach().mul_(coef)
    return total


class CheckOverflow:

    def __init__(self, param_groups=None, mpu=None, zero_reduce_scatter=False, deepspeed=None):
        self.params = [p for g in (param_groups or []) for p in (g if isinstance(g, list) else g["params"])]

    def check(self, param_groups=None):
        params = self.params if param_groups is None else [p for g in param_groups for p in g]
        return self.has_overflow(params)

    @staticmethod
    def has_overflow(params):
        flag = torch.zeros((), dtype=torch.int32, device=params[0].device if params else "cpu")
        for p in params:
            if p.grad is not None and not torch.isfinite(p.grad).all():
                flag.fill_(1)
                break
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return bool(flag.item())


def assert_ints_same_as_other_ranks(ints, group=None, what="values"):
    """Raise unless every rank of ``group`` passes the same list of ints (reference runtime/zero/utils.py:80-91,
    used by ZeRO ``safe_mode`` to catch ranks that disagree on parameter order or sizes before a collective
    silently mixes up their buffers)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    mine = [int(i) for i in ints]
    allv = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, mine, group=group)
    for r, v in enumerate(allv):
        if v != mine:
            raise RuntimeError(f"safe_mode: rank {dist.get_rank()} and group rank {r} disagree on {what}: "
                               f"{mine[:16]}... vs {v[:16]}...")


def see_memory_usage(message, force=False):
    if not force:
        return
    if dist.is_initialized() and dist.get_rank() != 0:
        return
    gc.collect()
    vm = psutil.virtual_memory()
    if torch.cuda.is_available():
        logger.info(f"{message} | MA {torch.cuda.memory_allocated() / 2**30:.2f} GB "
                    f"Max_MA {torch.cuda.max_memory_allocated() / 2**30:.2f} GB "
                    f"CA {torch.cuda.memory_reserved() / 2**30:.2f} GB "
                    f"Max_CA {torch.cuda.max_memory_reserved() / 2**30:.2f} GB")
        torch.cuda.reset_peak_memory_stats()
    logger.info(f"{message} | CPU Virtual Memory: used = {(vm.total - vm.available) / 2**30:.2f} GB, "
                f"percent = {vm.percent}%")


def all_gather_dp_groups(groups_flat, partitioned_param_groups, dp_process_group, start_alignment_factor=None,
                         allgather_bucket_size=None):
    """Rebuild full flat buffers from their data-parallel partitions (one all_gather_into_tensor each)."""
    for full, parts, g in zip(groups_flat, partitioned_param_groups, dp_process_group):
        mine = parts[dist.get_rank(g)]
        dist.all_gather_into_tensor(full, mine, group=g)


def call_to_str(base, *args, **kwargs):
    name = f"{base}("
    if args:
        name += ", ".join(repr(a) for a in args)
        if kwargs:
            name += ", "
    if kwargs:
        name += ", ".join(f"{k}={v!r}" for k, v in kwargs.items())
    return name + ")"


def graph_process(replay_first_step, func, *args, **kwargs):
    """Capture ``func`` into a HIP graph on the first call and replay it afterwards (reference :50-68).
    Returns (graph, outputs); callers keep the graph and call ``graph.replay()``."""
    if not torch.cuda.is_available():
        return None, func(*args, **kwargs)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        func(*args, **kwargs)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = func(*args, **kwargs)
    if replay_first_step:
        g.replay()
    return g, out


def empty_cache():
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
