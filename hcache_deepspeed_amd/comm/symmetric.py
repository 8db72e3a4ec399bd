"""Symmetric-memory collectives between the GPUs of one node (csrc/kernels/symm_comm.hip).

Reference parity: DeepCompile's ``symmetric_memory`` all-gather (csrc/compile/z3.cpp:91-110, compile config
``symmetric_memory``), and SURVEY.md §5.8's one-shot all-reduce for small collectives.

Every rank of ``group`` allocates one uncached device buffer (flags + two data slots of ``cap_bytes``), exports its
IPC handle, and maps every peer's buffer once. A collective is then ONE kernel on the caller's stream: each block
publishes its chunk into its own buffer, raises a per-block flag in every peer's buffer, waits for the peers'
flags and reads their chunks straight over xGMI -- no ring steps, no host involvement, all 7 links at once.

* ``all_reduce`` -- one-shot sum (fp32 accumulation, fixed rank order: bit-identical on every rank); the
  tensor-parallel all-reduce of decode-sized activations is its main user (inference v2, parallel/tp.py);
* ``all_gather_into_tensor`` / ``reduce_scatter_tensor`` -- direct-read variants, used by the ZeRO-3 unit
  collectives when ``compile.symmetric_memory`` is on (runtime/zero/optimizer.py ``enable_symmetric_comm``).

The protocol needs every rank to issue the same collectives of one ``SymmetricMemory`` in the same order on ONE
stream (like any collective); use separate objects for concurrently running streams. Waits inside the kernel are
bounded: a missing peer sets an error word (``error()``) instead of hanging the GPU.
"""
import ctypes
import os

import torch
import torch.distributed as dist

from ..ops import native

MAX_RANKS = 8
_cache = {}
# one-shot all-reduce threshold of the tensor-parallel paths (0: always torch.distributed / RCCL)
SMALL_ALLREDUCE_KB = int(os.environ.get("HDS_SYMM_ALLREDUCE_KB", "0"))


def supported(group=None):
    """Symmetric memory needs a GPU, an initialised process group of <= 8 ranks."""
    return torch.cuda.is_available() and dist.is_initialized() and 1 < dist.get_world_size(group) <= MAX_RANKS


class SymmetricMemory:

    def __init__(self, group=None, cap_bytes=16 << 20):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if not 1 <= self.world <= MAX_RANKS:
            raise ValueError(f"symmetric memory supports 1..{MAX_RANKS} ranks, got {self.world}")
        self.lib = native.kernels()
        self.cap = (int(cap_bytes) + 15) // 16 * 16
        ptr, handle = ctypes.c_void_p(), ctypes.create_string_buffer(64)
        native.check(self.lib.hds_symm_alloc(self.cap, ctypes.byref(ptr), handle), "symm_alloc")
        self._own = ptr.value
        handles = [None] * self.world
        dist.all_gather_object(handles, handle.raw, group=group)
        bases, self._opened = [], []
        for r, h in enumerate(handles):
            if r == self.rank:
                bases.append(self._own)
                continue
            p = ctypes.c_void_p()
            native.check(self.lib.hds_symm_open(h, ctypes.byref(p)), "symm_open")
            bases.append(p.value)
            self._opened.append(p.value)
        self._bases = (ctypes.c_int64 * MAX_RANKS)(*(bases + [0] * (MAX_RANKS - len(bases))))
        self.epoch = 0
        self.calls = {"all_reduce": 0, "all_gather": 0, "reduce_scatter": 0}

    def _next(self):
        self.epoch = (self.epoch + 1) & 0xFFFFFFFF or 1
        return self.epoch

    def fits(self, nbytes, align=16):
        return 0 < nbytes <= self.cap and nbytes % align == 0

    def all_reduce(self, t, out=None):
        """Sum of ``t`` over the group into ``out`` (default in place); returns ``out``."""
        out = t if out is None else out
        n = t.numel()
        if not (t.is_contiguous() and out.is_contiguous() and n % 8 == 0 and self.fits(n * t.element_size())):
            raise ValueError("symmetric all_reduce: contiguous, numel % 8 == 0 and within the buffer capacity")
        native.check(self.lib.hds_symm_allreduce(ctypes.addressof(self._bases), self.rank, self.world, self.cap,
                                                 self._next(), t.data_ptr(), out.data_ptr(), n, native.dt(t),
                                                 native.stream()), "symm_allreduce")
        self.calls["all_reduce"] += 1
        return out

    def all_gather_into_tensor(self, out, inp):
        nb = inp.numel() * inp.element_size()
        if not (inp.is_contiguous() and out.is_contiguous() and out.numel() == inp.numel() * self.world
                and self.fits(nb)):
            raise ValueError("symmetric all_gather: contiguous, out = world x inp, shard bytes % 16 within capacity")
        native.check(self.lib.hds_symm_allgather(ctypes.addressof(self._bases), self.rank, self.world, self.cap,
                                                 self._next(), inp.data_ptr(), out.data_ptr(), nb, native.stream()),
                     "symm_allgather")
        self.calls["all_gather"] += 1
        return out

    def reduce_scatter_tensor(self, out, inp):
        n = out.numel()
        if not (inp.is_contiguous() and out.is_contiguous() and inp.numel() == n * self.world and n % 8 == 0
                and self.fits(inp.numel() * inp.element_size()) and inp.dtype == out.dtype):
            raise ValueError("symmetric reduce_scatter: contiguous, inp = world x out, numel % 8, within capacity")
        native.check(self.lib.hds_symm_reduce_scatter(ctypes.addressof(self._bases), self.rank, self.world, self.cap,
                                                      self._next(), inp.data_ptr(), out.data_ptr(), n,
                                                      native.dt(inp), native.stream()), "symm_reduce_scatter")
        self.calls["reduce_scatter"] += 1
        return out

    def error(self):
        """0, or 1 + the peer whose flag never arrived (device read; synchronizes)."""
        return int(self.lib.hds_symm_error(ctypes.c_void_p(self._own)))

    def close(self):
        if self._own is None:
            return
        torch.cuda.synchronize()
        dist.barrier(group=self.group)  # no peer still reads this rank's buffer
        for p in self._opened:
            self.lib.hds_symm_close(ctypes.c_void_p(p))
        self._opened = []
        native.check(self.lib.hds_symm_free(ctypes.c_void_p(self._own)), "symm_free")
        self._own = None


def get_symmetric(group=None, cap_bytes=16 << 20, tag="default"):
    """Process-wide ``SymmetricMemory`` per (group, tag); every rank of the group must call it collectively."""
    key = (id(group), tag)
    sm = _cache.get(key)
    if sm is None or sm.cap < cap_bytes:
        if sm is not None:
            sm.close()
        sm = _cache[key] = SymmetricMemory(group, cap_bytes)
    return sm


def release_all():
    for sm in list(_cache.values()):
        sm.close()
    _cache.clear()


def small_all_reduce(x, group=None, max_kb=None):
    """In-place sum of ``x`` over ``group``: the one-shot symmetric all-reduce for contiguous GPU messages of at
    most ``max_kb`` KiB (default ``HDS_SYMM_ALLREDUCE_KB``) on a group of <= 8 ranks, RCCL otherwise. The choice
    depends only on the message size and the group, so every rank of a tensor-parallel group takes the same path."""
    kb = SMALL_ALLREDUCE_KB if max_kb is None else max_kb
    nb = x.numel() * x.element_size()
    if (kb > 0 and x.is_cuda and x.is_contiguous() and x.numel() % 8 == 0 and 0 < nb <= kb * 1024
            and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and supported(group)):
        get_symmetric(group, cap_bytes=kb * 1024, tag="small_allreduce").all_reduce(x)
        return x
    dist.all_reduce(x, group=group)
    return x
