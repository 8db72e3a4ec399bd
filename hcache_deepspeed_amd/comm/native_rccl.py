"""Native RCCL communicator (csrc/host/rccl_comm.cpp) — the C++ comm layer of SURVEY.md §5.8 / DeepCompile N20.

``RcclCommunicator(group)`` creates ONE private RCCL communicator for a ``torch.distributed`` group: rank 0 of the
group draws the unique id in C++, it is broadcast once over the existing process group, and every rank calls
``ncclCommInitRank`` on its current HIP device. The C++ side issues on a high-priority communication stream (from torch's
stream pool) and keeps a ring of completion events:

* every collective is ordered after the work queued on the caller's stream by a GPU-side event wait (no host sync),
* it runs on the private comm stream (so it overlaps compute queued later on the caller's stream),
* the returned :class:`Work` makes the caller's stream wait for it (``wait()``) — again on the GPU — or reports
  completion without blocking (``is_completed()``).

Tensors passed in are recorded on the comm stream (``record_stream``) so the caching allocator does not recycle
them while the collective is in flight. Used by ``engine.compile()``'s native-comm mode
(``"compile": {"native_comm": true}``) for the ZeRO all-gather / reduce-scatter; also usable directly.
"""
import ctypes
import os

import torch
import torch.distributed as tdist

from ..ops import native

_DT = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
       torch.float64: 8, torch.bfloat16: 9}
_OP = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


def _op(op):
    if isinstance(op, str):
        return _OP[op]
    name = str(op).split(".")[-1].lower()
    return _OP.get(name, 0)


def _lib():
    lib = native.host_lib()
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    rc = lib.hds_rccl_load(path.encode())
    if rc != 0:
        raise RuntimeError(f"native RCCL: cannot load {path} (code {rc})")
    return lib


class Work:
    """Completion handle of one native collective."""

    def __init__(self, comm, slot, keep):
        self._comm, self._slot, self._keep = comm, slot, keep

    def wait(self, stream=None):
        if self._comm._h is None:  # communicator destroyed: its stream was synchronized then
            return True
        s = stream or torch.cuda.current_stream()
        self._comm._check(self._comm._lib.hds_rccl_wait(self._comm._h, self._slot, ctypes.c_void_p(s.cuda_stream)),
                          "wait")
        self._keep = None
        return True

    def is_completed(self):
        if self._comm._h is None:
            return True
        return self._comm._lib.hds_rccl_query(self._comm._h, self._slot) == 1


_fail_setup_ranks = set()  # fault injection (tests): these ranks' local setup raises


class RcclCommunicator:

    def __init__(self, group=None):
        if not torch.cuda.is_available():
            raise RuntimeError("native RCCL communicator needs a GPU")
        self._lib = _lib()
        self.group = group
        self.rank = tdist.get_rank(group) if tdist.is_initialized() else 0
        self.world = tdist.get_world_size(group) if tdist.is_initialized() else 1
        from .setup import collective_setup
        # torch's pooled streams are never destroyed, so record_stream() events on it outlive this object
        self.stream = torch.cuda.Stream(priority=-1)
        self._h = None

        # failure-symmetric (comm/setup.py): rank 0's unique id travels in the same all_gather_object that agrees on
        # every rank's local readiness; the init result is agreed again, so a rank that failed never leaves the
        # others in a different collective
        def local():
            if _fail_setup_ranks and self.rank in _fail_setup_ranks:
                raise RuntimeError("injected native RCCL setup failure")
            uid = ctypes.create_string_buffer(128)
            if self.rank == 0:
                self._check(self._lib.hds_rccl_unique_id(uid), "unique_id")
            return None, (bytes(uid.raw) if self.rank == 0 else None)

        def finish(_, payloads):
            uid = ctypes.create_string_buffer(payloads[0], 128)
            err = ctypes.c_int(0)
            h = self._lib.hds_rccl_init(uid, self.world, self.rank, ctypes.c_void_p(self.stream.cuda_stream),
                                        ctypes.byref(err))
            if not h:
                raise RuntimeError(f"native RCCL init failed: {self._err(err.value)}")
            return h

        def cleanup(_, h):
            if h:
                self._lib.hds_rccl_destroy(h)

        _, self._h = collective_setup(group, local, finish, cleanup, what="native RCCL communicator")

    def _err(self, rc):
        s = self._lib.hds_rccl_error_string(rc)
        return s.decode() if s else str(rc)

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"native RCCL {what} failed: {self._err(rc)}")

    def _issue(self, fn, what, tensors, *args):
        caller = torch.cuda.current_stream()
        slot = ctypes.c_int(0)
        self._check(fn(self._h, *args, ctypes.c_void_p(caller.cuda_stream), ctypes.byref(slot)), what)
        for t in tensors:
            t.record_stream(self.stream)
        return Work(self, slot.value, tensors)

    @staticmethod
    def _dt(t):
        if t.dtype not in _DT:
            raise TypeError(f"native RCCL: unsupported dtype {t.dtype}")
        return _DT[t.dtype]

    def all_gather_into_tensor(self, out, inp, async_op=False):
        assert out.numel() == inp.numel() * self.world and out.is_contiguous() and inp.is_contiguous()
        w = self._issue(self._lib.hds_rccl_all_gather, "all_gather", (out, inp), ctypes.c_void_p(inp.data_ptr()),
                        ctypes.c_void_p(out.data_ptr()), inp.numel(), self._dt(inp))
        return w if async_op else w.wait()

    def reduce_scatter_tensor(self, out, inp, op="sum", async_op=False):
        assert inp.numel() == out.numel() * self.world and out.is_contiguous() and inp.is_contiguous()
        w = self._issue(self._lib.hds_rccl_reduce_scatter, "reduce_scatter", (out, inp),
                        ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()), out.numel(), self._dt(inp),
                        _op(op))
        return w if async_op else w.wait()

    def all_reduce(self, t, op="sum", async_op=False):
        assert t.is_contiguous()
        w = self._issue(self._lib.hds_rccl_all_reduce, "all_reduce", (t, ), ctypes.c_void_p(t.data_ptr()),
                        ctypes.c_void_p(t.data_ptr()), t.numel(), self._dt(t), _op(op))
        return w if async_op else w.wait()

    def broadcast(self, t, root=0, async_op=False):
        assert t.is_contiguous()
        w = self._issue(self._lib.hds_rccl_broadcast, "broadcast", (t, ), ctypes.c_void_p(t.data_ptr()),
                        ctypes.c_void_p(t.data_ptr()), t.numel(), self._dt(t), root)
        return w if async_op else w.wait()

    def all_to_all_single(self, out, inp, async_op=False):
        assert out.numel() == inp.numel() and inp.numel() % self.world == 0
        w = self._issue(self._lib.hds_rccl_all_to_all, "all_to_all", (out, inp), ctypes.c_void_p(inp.data_ptr()),
                        ctypes.c_void_p(out.data_ptr()), inp.numel() // self.world, self._dt(inp),
                        inp.element_size())
        return w if async_op else w.wait()

    def synchronize(self):
        self._check(self._lib.hds_rccl_synchronize(self._h), "synchronize")

    def destroy(self):
        """Free the RCCL communicator (collective: every rank of the group must call it). Not done implicitly:
        a destructor running at interpreter teardown could block on peers that already exited."""
        if getattr(self, "_h", None):
            self._lib.hds_rccl_destroy(self._h)
            self._h = None
