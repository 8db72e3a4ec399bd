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
stream (like any collective); use separate objects for concurrently running streams.

Failure is loud, never silent: waits inside the kernel are bounded, and a timed-out wait (a peer that fell behind by
more than the bound, or never issued the collective) marks the buffer failed for good. The kernel writes the error to
a host-mapped pinned status word that every later call checks for free (``SymmetricMemoryError`` is raised, and the
group is marked broken so ``small_all_reduce`` falls back to RCCL), and to an optional device flag (``dev_status``)
that the ZeRO optimizer folds into its step-skip flag, so the step that consumed stale peer data does not update the
weights (runtime/zero/optimizer.py).
"""
import ctypes
import os

import torch
import torch.distributed as dist

from ..ops import native

MAX_RANKS = 8
_cache = {}
_broken = set()  # (id(group), tag) of buffers that timed out: RCCL from then on
# one-shot all-reduce threshold of the tensor-parallel paths (0: always torch.distributed / RCCL). Decode-sized
# all-reduces (<= 256 KiB: [batch, hidden] activations) are latency-bound, where one kernel reading all peers over
# every xGMI link beats a ring's 2(W-1) steps
SMALL_ALLREDUCE_KB = int(os.environ.get("HDS_SYMM_ALLREDUCE_KB", "256"))


class SymmetricMemoryError(RuntimeError):
    """A symmetric-memory collective timed out waiting for a peer: results since then are not trustworthy."""


_same_node = {}  # id(group) -> every rank of the group runs on this host
_fail_setup_ranks = set()  # fault injection (tests): these ranks' local setup raises


def _host_id():
    """This host's identity: hostname + kernel boot id (containers of different machines may share a hostname)."""
    import socket
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return f"{socket.gethostname()}/{boot}"


def same_node(group=None):
    """True iff every rank of ``group`` runs on this host (IPC handles do not cross nodes). Collective the first time
    per group (an all_gather_object of the host ids), cached after."""
    key = id(group)
    if key not in _same_node:
        ids = [None] * dist.get_world_size(group)
        dist.all_gather_object(ids, _host_id(), group=group)
        _same_node[key] = len(set(ids)) == 1
    return _same_node[key]


def supported(group=None):
    """Symmetric memory needs a GPU and an initialised process group of <= 8 ranks, all on this node. Collective
    (``same_node``): every rank of the group must call it."""
    return (torch.cuda.is_available() and dist.is_initialized() and 1 < dist.get_world_size(group) <= MAX_RANKS
            and same_node(group))


class SymmetricMemory:

    def __init__(self, group=None, cap_bytes=16 << 20):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if not 1 <= self.world <= MAX_RANKS:
            raise ValueError(f"symmetric memory supports 1..{MAX_RANKS} ranks, got {self.world}")
        self.cap = (int(cap_bytes) + 15) // 16 * 16
        self._own, self._opened, self._status = None, [], None
        from .setup import collective_setup

        # three failure-symmetric phases (comm/setup.py): local allocation, ONE all_gather_object that both agrees
        # and exchanges the IPC handles, then opening the peers' buffers with a second agreement -- a rank whose
        # allocation fails (OOM) can no longer leave its peers waiting in a different collective
        def local():
            if _fail_setup_ranks and self.rank in _fail_setup_ranks:
                raise RuntimeError("injected symmetric-memory setup failure")
            lib = native.kernels()
            ptr, handle = ctypes.c_void_p(), ctypes.create_string_buffer(64)
            native.check(lib.hds_symm_alloc(self.cap, ctypes.byref(ptr), handle), "symm_alloc")
            st = ctypes.c_void_p()
            if lib.hds_symm_status_alloc(ctypes.byref(st)) != 0:
                lib.hds_symm_free(ptr)
                raise RuntimeError("symm_status_alloc failed")
            return (lib, ptr.value, st.value), handle.raw

        def finish(state, handles):
            lib, own, _ = state
            bases, opened = [], []
            try:
                for r, h in enumerate(handles):
                    if r == self.rank:
                        bases.append(own)
                        continue
                    p = ctypes.c_void_p()
                    native.check(lib.hds_symm_open(h, ctypes.byref(p)), "symm_open")
                    bases.append(p.value)
                    opened.append(p.value)
            except Exception:
                for q in opened:
                    lib.hds_symm_close(ctypes.c_void_p(q))
                raise
            return bases, opened

        def cleanup(state, fin):
            if state is None:
                return
            lib, own, st = state
            for q in (fin[1] if fin else []):
                lib.hds_symm_close(ctypes.c_void_p(q))
            lib.hds_symm_free(ctypes.c_void_p(own))
            lib.hds_symm_status_free(ctypes.c_void_p(st))

        (self.lib, self._own, self._status), (bases, self._opened) = collective_setup(
            group, local, finish, cleanup, what=f"symmetric memory ({self.cap >> 20} MiB)")
        self._bases = (ctypes.c_int64 * MAX_RANKS)(*(bases + [0] * (MAX_RANKS - len(bases))))
        self._status_word = ctypes.c_uint32.from_address(self._status)
        self.epoch = 0
        self.calls = {"all_reduce": 0, "all_gather": 0, "reduce_scatter": 0}

    def _next(self):
        self.epoch = (self.epoch + 1) & 0xFFFFFFFF or 1
        return self.epoch

    def fits(self, nbytes, align=16):
        return 0 < nbytes <= self.cap and nbytes % align == 0

    def error_nowait(self):
        """0, or the error code a completed collective of this buffer reported (a host-memory read: no sync)."""
        return int(self._status_word.value)

    def check(self):
        """Raise ``SymmetricMemoryError`` if any completed collective of this buffer timed out."""
        e = self.error_nowait()
        if e:
            what = (f"peer {(e & 0xFF) - 1} timed out and poisoned this buffer" if e & 0x100 else
                    f"timed out waiting for peer {e - 1}")
            raise SymmetricMemoryError(f"symmetric-memory collective on rank {self.rank}: {what} (world {self.world}); "
                                       f"results of this buffer since then are invalid")

    @staticmethod
    def _dev(dev_status):
        if dev_status is None:
            return None
        assert dev_status.is_cuda and dev_status.dtype == torch.int32
        return dev_status.data_ptr()

    def all_reduce(self, t, out=None, dev_status=None, check=True):
        """Sum of ``t`` over the group into ``out`` (default in place); returns ``out``. ``check``: raise first if an
        earlier collective of this buffer timed out (callers that fold ``dev_status`` into a step flag pass False)."""
        if check:
            self.check()
        out = t if out is None else out
        n = t.numel()
        if not (t.is_contiguous() and out.is_contiguous() and n % 8 == 0 and self.fits(n * t.element_size())):
            raise ValueError("symmetric all_reduce: contiguous, numel % 8 == 0 and within the buffer capacity")
        native.check(self.lib.hds_symm_allreduce(ctypes.addressof(self._bases), self.rank, self.world, self.cap,
                                                 self._next(), t.data_ptr(), out.data_ptr(), n, native.dt(t),
                                                 self._status, self._dev(dev_status), native.stream()),
                     "symm_allreduce")
        self.calls["all_reduce"] += 1
        return out

    def all_gather_into_tensor(self, out, inp, dev_status=None, check=True):
        if check:
            self.check()
        nb = inp.numel() * inp.element_size()
        if not (inp.is_contiguous() and out.is_contiguous() and out.numel() == inp.numel() * self.world
                and self.fits(nb)):
            raise ValueError("symmetric all_gather: contiguous, out = world x inp, shard bytes % 16 within capacity")
        native.check(self.lib.hds_symm_allgather(ctypes.addressof(self._bases), self.rank, self.world, self.cap,
                                                 self._next(), inp.data_ptr(), out.data_ptr(), nb, self._status,
                                                 self._dev(dev_status), native.stream()), "symm_allgather")
        self.calls["all_gather"] += 1
        return out

    def reduce_scatter_tensor(self, out, inp, dev_status=None, check=True):
        if check:
            self.check()
        n = out.numel()
        if not (inp.is_contiguous() and out.is_contiguous() and inp.numel() == n * self.world and n % 8 == 0
                and self.fits(inp.numel() * inp.element_size()) and inp.dtype == out.dtype):
            raise ValueError("symmetric reduce_scatter: contiguous, inp = world x out, numel % 8, within capacity")
        native.check(self.lib.hds_symm_reduce_scatter(ctypes.addressof(self._bases), self.rank, self.world, self.cap,
                                                      self._next(), inp.data_ptr(), out.data_ptr(), n,
                                                      native.dt(inp), self._status, self._dev(dev_status),
                                                      native.stream()), "symm_reduce_scatter")
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
        self.lib.hds_symm_status_free(ctypes.c_void_p(self._status))
        self._status, self._status_word = None, ctypes.c_uint32(0)

    def abandon(self):
        """Drop a failed buffer WITHOUT the collective barrier of ``close`` (a peer may be gone); the IPC mappings
        and the allocation are released at process exit."""
        self._own = None
        self._opened = []


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


def _agree_broken(group):
    """Called by a rank whose buffer failed. The failing rank poisoned every peer's buffer (symm_comm.hip), so each
    peer fails its next symmetric call too and arrives here: the ranks meet in one torch.distributed collective and
    only then switch the group to RCCL together -- never one rank on RCCL while another still waits in the symmetric
    protocol. The agreement is a MAX of 1 over the group (host tensor on gloo)."""
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    flag = torch.ones(1, dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    _broken.add((id(group), "small_allreduce"))


def small_all_reduce(x, group=None, max_kb=None):
    """In-place sum of ``x`` over ``group``: the one-shot symmetric all-reduce for contiguous GPU messages of at
    most ``max_kb`` KiB (default ``HDS_SYMM_ALLREDUCE_KB``) on a group of <= 8 ranks on one node, RCCL otherwise. The
    choice depends only on the message size and the group, so every rank of a tensor-parallel group takes the same
    path; after a timeout the switch to RCCL is agreed collectively (``_agree_broken``) and the call raises."""
    kb = SMALL_ALLREDUCE_KB if max_kb is None else max_kb
    nb = x.numel() * x.element_size()
    if (kb > 0 and x.is_cuda and x.is_contiguous() and x.numel() % 8 == 0 and 0 < nb <= kb * 1024
            and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and supported(group)
            and (id(group), "small_allreduce") not in _broken):
        sm = get_symmetric(group, cap_bytes=kb * 1024, tag="small_allreduce")
        try:
            sm.all_reduce(x)
        except SymmetricMemoryError:
            # loud: the caller's earlier results may be stale; once every rank of the group has failed too (the
            # poison makes sure they do), later calls of this group take RCCL on every rank
            _agree_broken(group)
            _cache.pop((id(group), "small_allreduce"), None)
            sm.abandon()
            raise
        return x
    dist.all_reduce(x, group=group)
    return x
