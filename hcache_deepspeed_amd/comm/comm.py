"""``deepspeed.comm``-compatible collective facade over torch.distributed (RCCL on GPU, gloo on CPU).

Reference parity: deepspeed/comm/comm.py (module-level torch.distributed mirror with ``@timed_op``
logging, init_distributed :636-702, env discovery :705-808) and comm/torch.py (TorchBackend).

MI355X notes:
* the GPU backend is ``"nccl"`` which IS RCCL on ROCm; one process per GPU;
* ZeRO never issues list-form collectives: only flat ``all_gather_into_tensor`` /
  ``reduce_scatter_tensor`` over rank-major buffers (see runtime/zero/flat.py), which map onto
  RCCL's xGMI ring/direct kernels without per-tensor launches;
* ``new_group`` is used to create *separate* communicators for the all-gather (prefetch) and the
  reduce-scatter (gradient) traffic of ZeRO-3 so the two directions overlap instead of serializing
  on one RCCL stream.
"""
import functools
import os
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from ..utils.comms_logging import CommsLogger, msg_bytes
from ..utils.logging import logger

ReduceOp = dist.ReduceOp

DEFAULT_TIMEOUT_MIN = int(os.environ.get("DEEPSPEED_TIMEOUT", 30))
comms_logger = CommsLogger()
_local_rank = None


# -----------------------------------------------------------------------------------------
# timed_op: latency / algbw / busbw per collective when the comms logger is enabled
# -----------------------------------------------------------------------------------------
def timed_op(func):

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        if not comms_logger.enabled or kwargs.get("async_op", False):
            return func(*args, **kwargs)
        prof = kwargs.pop("prof", False)
        log_name = kwargs.pop("log_name", func.__name__)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = func(*args, **kwargs)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        lat = (time.perf_counter() - t0) * 1e3
        size = msg_bytes(func.__name__, args, kwargs)
        group = kwargs.get("group")
        comms_logger.append(func.__name__, log_name, lat, size, get_world_size(group))
        return out

    return wrapper


def configure(ds_config=None, enabled=None, prof_all=None, prof_ops=None, verbose=None, debug=None):
    if ds_config is not None and getattr(ds_config, "comms_logger", None) is not None:
        c = ds_config.comms_logger
        comms_logger.configure(c.get("enabled", False), c.get("prof_all", True), c.get("prof_ops", []),
                               c.get("verbose", False), c.get("debug", False))
    if enabled is not None:
        comms_logger.enabled = enabled
    if prof_all is not None:
        comms_logger.prof_all = prof_all
    if prof_ops is not None:
        comms_logger.prof_ops = prof_ops
    if verbose is not None:
        comms_logger.verbose = verbose


def log_summary(show_straggler=False):
    barrier()
    if get_rank() == 0:
        comms_logger.log_all()
    barrier()


# -----------------------------------------------------------------------------------------
# init
# -----------------------------------------------------------------------------------------
def is_available():
    return dist.is_available()


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def _discover_env(verbose=True):
    """Fill RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* from MPI / SLURM variables when torchrun did not."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return
    for rk, ws, lr in (("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),
                       ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"), ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID")):
        if rk in os.environ:
            os.environ["RANK"] = os.environ[rk]
            os.environ["WORLD_SIZE"] = os.environ[ws]
            os.environ["LOCAL_RANK"] = os.environ.get(lr, "0")
            break
    else:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if verbose:
        logger.info(f"env discovery: RANK={os.environ['RANK']} WORLD_SIZE={os.environ['WORLD_SIZE']}")


def default_backend():
    return "nccl" if torch.cuda.is_available() else "gloo"


def init_distributed(dist_backend=None, auto_mpi_discovery=True, distributed_port=29500, verbose=True,
                     timeout=timedelta(minutes=DEFAULT_TIMEOUT_MIN), init_method=None, dist_init_required=None,
                     config=None, rank=-1, world_size=-1):
    """Initialise torch.distributed (idempotent). Backend: nccl(=RCCL) on GPU, gloo on CPU."""
    global _local_rank
    if config is not None:
        configure(config)
    if is_initialized():
        return
    if dist_init_required is False:
        return
    if auto_mpi_discovery and rank < 0:
        _discover_env(verbose=verbose)
    os.environ.setdefault("MASTER_PORT", str(distributed_port))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = dist_backend or default_backend()
    if rank < 0:
        rank = int(os.environ.get("RANK", 0))
    if world_size < 0:
        world_size = int(os.environ.get("WORLD_SIZE", 1))
    _local_rank = int(os.environ.get("LOCAL_RANK", rank))
    kwargs = dict(backend=backend, rank=rank, world_size=world_size, timeout=timeout)
    if init_method:
        kwargs["init_method"] = init_method
    if backend == "nccl" and torch.cuda.is_available():
        torch.cuda.set_device(_local_rank % max(1, torch.cuda.device_count()))
        kwargs["device_id"] = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(**kwargs)
    if verbose and rank == 0:
        logger.info(f"initialized torch.distributed backend={backend} world_size={world_size}")


def destroy_process_group(group=None):
    if is_initialized():
        dist.destroy_process_group(group)


def get_rank(group=None):
    return dist.get_rank(group) if is_initialized() else 0


def get_world_size(group=None):
    return dist.get_world_size(group) if is_initialized() else 1


def get_local_rank():
    if _local_rank is not None:
        return _local_rank
    return int(os.environ.get("LOCAL_RANK", 0))


def get_global_rank(group, group_rank):
    if group is None:
        return group_rank
    return dist.get_global_rank(group, group_rank)


def get_world_group():
    return dist.group.WORLD


def get_backend(group=None):
    return dist.get_backend(group) if is_initialized() else None


def new_group(ranks=None, high_priority=False, **kwargs):
    """``high_priority``: with RCCL, the group's collectives run on high-priority HIP streams
    (``ProcessGroupNCCL.Options.is_high_priority_stream``) so they are dispatched ahead of queued compute."""
    if not is_initialized():
        return None
    if high_priority and "pg_options" not in kwargs and get_backend() == "nccl":
        opts = getattr(dist, "ProcessGroupNCCL", None)
        if opts is not None:
            o = opts.Options()
            o.is_high_priority_stream = True
            kwargs["pg_options"] = o
    return dist.new_group(ranks=ranks, **kwargs)


def supports_avg(group=None):
    return get_backend(group) == "nccl"


# -----------------------------------------------------------------------------------------
# collectives (world_size==1 short-circuits keep single-GPU runs free of RCCL launches)
# -----------------------------------------------------------------------------------------
class _Done:
    """Completed-work handle for short-circuited collectives."""

    def wait(self):
        return True

    def is_completed(self):
        return True


def _single(group):
    return get_world_size(group) == 1


# Debug switches that turn whole collective families into no-ops (reference comm/torch.py:58-93): used to
# measure how much of a step is communication-bound without changing the program.
_OFF = {"all_gather": False, "reduce_scatter": False, "broadcast": False, "all_reduce": False, "reduce": False}


def all_gather_comm_off(flag=False):
    _OFF["all_gather"] = bool(flag)


def reduce_scatter_comm_off(flag=False):
    _OFF["reduce_scatter"] = bool(flag)


def broadcast_comm_off(flag=False):
    _OFF["broadcast"] = bool(flag)


def all_reduce_comm_off(flag=False):
    _OFF["all_reduce"] = bool(flag)


def reduce_comm_off(flag=False):
    _OFF["reduce"] = bool(flag)


def backward_comm_off(flag=False):
    all_gather_comm_off(flag)
    reduce_scatter_comm_off(flag)


@timed_op
def all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False, prof=False, log_name="all_reduce"):
    if _OFF["all_reduce"] and not _single(group):
        return _Done() if async_op else None
    if _single(group):
        return _Done() if async_op else None
    return dist.all_reduce(tensor, op=op, group=group, async_op=async_op)


@timed_op
def inference_all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False):
    """TP inference all-reduce: CPU fp32/bf16 tensors of single-host jobs go through the shared-memory
    all-reduce (csrc/host/shm_comm.cpp, reference csrc/cpu/comm/shm.cpp); everything else uses the
    process group (RCCL on GPU)."""
    if op == ReduceOp.SUM and not _single(group):
        from .shm import get_shm_comm, shm_eligible
        if shm_eligible(tensor, group):
            get_shm_comm(group).all_reduce_(tensor)
            return _Done() if async_op else None
    return all_reduce(tensor, op=op, group=group, async_op=async_op)


@timed_op
def all_reduce_coalesced(tensors, op=ReduceOp.SUM, group=None, async_op=False):
    if _single(group):
        return _Done() if async_op else None
    flat = torch.cat([t.reshape(-1) for t in tensors])
    w = dist.all_reduce(flat, op=op, group=group, async_op=False)
    off = 0
    for t in tensors:
        t.copy_(flat[off:off + t.numel()].view_as(t))
        off += t.numel()
    return _Done() if async_op else w


@timed_op
def all_gather_coalesced(output_tensors, input_tensors, group=None, async_op=False):
    """All-gather a list of tensors with ONE collective: inputs are packed into one flat buffer, gathered
    rank-major with ``all_gather_into_tensor`` and unpacked into ``output_tensors[i]`` (each ``world`` times the
    size of ``input_tensors[i]``, rank-major)."""
    world = get_world_size(group)
    if _single(group):
        for o, i in zip(output_tensors, input_tensors):
            o.view(-1)[:i.numel()].copy_(i.reshape(-1))
        return _Done() if async_op else None
    if _OFF["all_gather"]:
        return _Done() if async_op else None
    sizes = [t.numel() for t in input_tensors]
    flat = torch.cat([t.reshape(-1) for t in input_tensors])
    out = torch.empty(world * flat.numel(), dtype=flat.dtype, device=flat.device)
    dist.all_gather_into_tensor(out, flat, group=group)
    out = out.view(world, -1)
    off = 0
    for o, n in zip(output_tensors, sizes):
        o.view(world, n).copy_(out[:, off:off + n])
        off += n
    return _Done() if async_op else None


@timed_op
def reduce(tensor, dst, op=ReduceOp.SUM, group=None, async_op=False):
    if _OFF["reduce"] and not _single(group):
        return _Done() if async_op else None
    if _single(group):
        return _Done() if async_op else None
    return dist.reduce(tensor, dst, op=op, group=group, async_op=async_op)


@timed_op
def broadcast(tensor, src, group=None, async_op=False):
    if _OFF["broadcast"] and not _single(group):
        return _Done() if async_op else None
    if _single(group):
        return _Done() if async_op else None
    return dist.broadcast(tensor, src, group=group, async_op=async_op)


def broadcast_object_list(object_list, src=0, group=None, device=None):
    if _single(group):
        return
    return dist.broadcast_object_list(object_list, src=src, group=group, device=device)


def all_gather_object(object_list, obj, group=None):
    if _single(group):
        object_list[0] = obj
        return
    return dist.all_gather_object(object_list, obj, group=group)


@timed_op
def all_gather(tensor_list, tensor, group=None, async_op=False):
    if _OFF["all_gather"] and not _single(group):
        return _Done() if async_op else None
    if _single(group):
        tensor_list[0].copy_(tensor)
        return _Done() if async_op else None
    return dist.all_gather(tensor_list, tensor, group=group, async_op=async_op)


@timed_op
def all_gather_into_tensor(output_tensor, tensor, group=None, async_op=False):
    if _OFF["all_gather"] and not _single(group):
        return _Done() if async_op else None
    if _single(group):
        if output_tensor.data_ptr() != tensor.data_ptr():
            output_tensor.copy_(tensor.view_as(output_tensor))
        return _Done() if async_op else None
    return dist.all_gather_into_tensor(output_tensor, tensor, group=group, async_op=async_op)


allgather_fn = all_gather_into_tensor


@timed_op
def reduce_scatter_tensor(output_tensor, tensor, op=ReduceOp.SUM, group=None, async_op=False):
    if _OFF["reduce_scatter"] and not _single(group):
        return _Done() if async_op else None
    if _single(group):
        if output_tensor.data_ptr() != tensor.data_ptr():
            output_tensor.copy_(tensor.view_as(output_tensor))
        return _Done() if async_op else None
    if op == ReduceOp.AVG and not supports_avg(group):
        w = dist.reduce_scatter_tensor(output_tensor, tensor, op=ReduceOp.SUM, group=group, async_op=False)
        output_tensor.div_(get_world_size(group))
        return _Done() if async_op else w
    return dist.reduce_scatter_tensor(output_tensor, tensor, op=op, group=group, async_op=async_op)


reduce_scatter_fn = reduce_scatter_tensor


@timed_op
def reduce_scatter(output, input_list, op=ReduceOp.SUM, group=None, async_op=False):
    if _OFF["reduce_scatter"] and not _single(group):
        return _Done() if async_op else None
    if _single(group):
        output.copy_(input_list[0])
        return _Done() if async_op else None
    return dist.reduce_scatter(output, input_list, op=op, group=group, async_op=async_op)


@timed_op
def all_to_all_single(output, tensor, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
    if _single(group):
        output.copy_(tensor)
        return _Done() if async_op else None
    return dist.all_to_all_single(output, tensor, output_split_sizes=output_split_sizes,
                                  input_split_sizes=input_split_sizes, group=group, async_op=async_op)


@timed_op
def all_to_all(output_tensor_list, input_tensor_list, group=None, async_op=False):
    if _single(group):
        output_tensor_list[0].copy_(input_tensor_list[0])
        return _Done() if async_op else None
    return dist.all_to_all(output_tensor_list, input_tensor_list, group=group, async_op=async_op)


@timed_op
def send(tensor, dst, group=None, tag=0):
    return dist.send(tensor, dst, group=group, tag=tag)


@timed_op
def recv(tensor, src=None, group=None, tag=0):
    return dist.recv(tensor, src, group=group, tag=tag)


def isend(tensor, dst, group=None, tag=0):
    return dist.isend(tensor, dst, group=group, tag=tag)


def irecv(tensor, src=None, group=None, tag=0):
    return dist.irecv(tensor, src, group=group, tag=tag)


def batch_isend_irecv(p2p_op_list):
    return dist.batch_isend_irecv(p2p_op_list)


P2POp = dist.P2POp


@timed_op
def gather(tensor, gather_list=None, dst=0, group=None, async_op=False):
    if _single(group):
        if gather_list is not None:
            gather_list[0].copy_(tensor)
        return _Done() if async_op else None
    return dist.gather(tensor, gather_list, dst, group=group, async_op=async_op)


@timed_op
def scatter(tensor, scatter_list=None, src=0, group=None, async_op=False):
    if _single(group):
        if scatter_list is not None:
            tensor.copy_(scatter_list[0])
        return _Done() if async_op else None
    return dist.scatter(tensor, scatter_list, src, group=group, async_op=async_op)


def barrier(group=None, async_op=False, device_ids=None):
    if not is_initialized() or get_world_size(group) == 1:
        return None
    if get_backend(group) == "nccl" and device_ids is None and torch.cuda.is_available():
        device_ids = [torch.cuda.current_device()]
    return dist.barrier(group=group, async_op=async_op, device_ids=device_ids)


def monitored_barrier(group=None, timeout=None, wait_all_ranks=False):
    if not is_initialized() or get_world_size(group) == 1:
        return None
    if get_backend(group) == "gloo":
        return dist.monitored_barrier(group=group, timeout=timeout, wait_all_ranks=wait_all_ranks)
    return barrier(group)


def initialize_mesh_device(mesh_shape, mesh_dim_names):
    from torch.distributed.device_mesh import init_device_mesh
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    return init_device_mesh(dev, mesh_shape, mesh_dim_names=mesh_dim_names)


def get_all_ranks_from_group(group=None):
    """Global ranks that make up ``group`` (reference comm.py:594)."""
    if group is None or not is_initialized():
        return list(range(get_world_size()))
    return dist.get_process_group_ranks(group)


def has_all_gather_into_tensor():
    return hasattr(dist, "all_gather_into_tensor")


def has_reduce_scatter_tensor():
    return hasattr(dist, "reduce_scatter_tensor")


def has_all_reduce_coalesced():
    return True


def has_coalescing_manager():
    return hasattr(dist.distributed_c10d, "_coalescing_manager")


def coalescing_manager(group=None, device=None, async_ops=False):
    """Batch the collectives issued inside the ``with`` block into one RCCL group launch (torch's
    ``_coalescing_manager``); a plain no-op context when unavailable or for a world of one."""
    import contextlib
    if not is_initialized() or _single(group) or not has_coalescing_manager():
        return contextlib.nullcontext()
    return dist.distributed_c10d._coalescing_manager(group, device=device, async_ops=async_ops)


def enable_symm_mem_for_group(group_name):
    """Reference comm.py:624 enables torch symmetric memory (CUDA multicast/NVLS). xGMI has no multicast object;
    RCCL already uses direct peer writes inside a node, so this is a logged no-op that reports False."""
    logger.info(f"symmetric memory not used on MI355X (group {group_name}): RCCL peer-to-peer over xGMI instead")
    return False
