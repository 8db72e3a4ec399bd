"""Debug helpers (reference utils/debug.py :14-153): module / parameter naming for ZeRO debugging, rank-locked
printing, per-rank log files and autograd-graph dumps."""
import fcntl

import torch

module_names = {}
param_names = {}


def debug_clear_module_and_param_names():
    module_names.clear()
    param_names.clear()


def debug_extract_module_and_param_names(model):
    module_names.update({m: n for n, m in model.named_modules()})
    param_names.update({p: n for n, p in model.named_parameters()})


def debug_module2name(module):
    return module_names.get(module, "unknown")


def debug_module2name_id(module):
    return f"name={debug_module2name(module)} id={getattr(module, 'id', None)}"


def debug_module2name_class(module):
    return f"name={debug_module2name(module)} {module.__class__.__name__}"


def debug_param2name(param):
    return param_names.get(param, "unknown")


def debug_param2name_id(param):
    return f"name={debug_param2name(param)} id={getattr(param, 'ds_id', None)}"


def debug_param2name_id_shape(param):
    return f"name={debug_param2name(param)} id={getattr(param, 'ds_id', None)} shape={tuple(param.shape)}"


def debug_param2name_id_shape_device(param):
    return (f"name={debug_param2name(param)} id={getattr(param, 'ds_id', None)} shape={tuple(param.shape)} "
            f"device={param.device}")


def debug_param2name_id_numel(param):
    return f"name={debug_param2name(param)} id={getattr(param, 'ds_id', None)} numel={param.numel()}"


def debug_param2name_id_shape_status(param):
    return (f"name={debug_param2name(param)} id={getattr(param, 'ds_id', None)} shape={tuple(param.shape)} "
            f"status={getattr(param, 'ds_status', None)}")


def printflock(*msgs):
    """Print under an exclusive file lock so multi-rank output does not interleave."""
    with open(__file__, "r") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            print(*msgs, flush=True)
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)


_rank_fh = {}


def log_rank_file(rank, *msgs):
    """Append to ``log_rank_{rank}.txt`` (one file per rank, for diffing ranks' behaviour)."""
    if rank not in _rank_fh:
        _rank_fh[rank] = open(f"log_rank_{rank}.txt", "w")
    fh = _rank_fh[rank]
    for m in msgs:
        fh.write(f"{m}\n")
    fh.flush()


def print_backward_tensors(tensor):
    """Walk the autograd graph below ``tensor``; print each node and the leaves it reaches."""

    def _walk(fn, depth=0):
        if fn is None:
            return
        print(" " * depth + type(fn).__name__)
        var = getattr(fn, "variable", None)
        if isinstance(var, torch.Tensor):
            print(" " * depth + f"  leaf {tuple(var.shape)} grad={'set' if var.grad is not None else None}")
        for nxt, _ in getattr(fn, "next_functions", ()):
            _walk(nxt, depth + 1)

    _walk(tensor.grad_fn)
