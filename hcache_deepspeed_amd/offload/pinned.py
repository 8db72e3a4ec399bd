"""Pinned host memory: hipHostMalloc buffers exposed as torch tensors, a slot ring, and a reuse pool.

Backed by csrc/host/pinned_ring.cpp. Host tensors created here alias the pinned allocation
(zero-copy ``torch.frombuffer`` over the hipHostMalloc pointer), so ``tensor.copy_(..., non_blocking=True)``
from/to the GPU runs as a true async DMA on whatever HIP stream is current.
"""
import ctypes
import threading

import torch

from ..ops import native

PORTABLE, MAPPED, WRITE_COMBINED = 1, 2, 4


class PinnedBuffer:
    """One hipHostMalloc allocation viewed as a torch tensor (freed with the object)."""

    def __init__(self, nbytes, flags=PORTABLE):
        self.nbytes = int(nbytes)
        self._lib = native.host_lib()
        self.ptr = self._lib.hds_host_alloc(self.nbytes, flags)
        if not self.ptr:
            raise MemoryError(f"hipHostMalloc({self.nbytes}) failed")
        arr = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        self._u8 = torch.frombuffer(arr, dtype=torch.uint8)

    def view(self, dtype, numel=None, offset_bytes=0):
        es = torch.tensor([], dtype=dtype).element_size()
        numel = numel if numel is not None else (self.nbytes - offset_bytes) // es
        return self._u8[offset_bytes:offset_bytes + numel * es].view(dtype)

    def __del__(self):
        try:
            if self.ptr:
                self._lib.hds_host_free(self.ptr)
                self.ptr = None
        except Exception:
            pass


def pinned_empty(shape, dtype, fast=False):
    """Pinned host tensor of ``shape`` (fast=True: portable|mapped|write-combined, the reference's fast host buffer)."""
    numel = 1
    for s in (shape if isinstance(shape, (tuple, list)) else (shape, )):
        numel *= int(s)
    es = torch.tensor([], dtype=dtype).element_size()
    buf = PinnedBuffer(max(1, numel * es), (PORTABLE | MAPPED | WRITE_COMBINED) if fast else PORTABLE)
    t = buf.view(dtype, numel).view(shape)
    t._hds_pinned_owner = buf  # keep the allocation alive with the tensor
    return t


class PinnedRing:
    """N fixed pinned slots with per-slot HIP events (acquire waits for the slot's previous transfer)."""

    def __init__(self, slot_bytes, nslots, flags=PORTABLE):
        self._lib = native.host_lib()
        self.h = self._lib.hds_ring_create(int(slot_bytes), int(nslots), flags)
        if not self.h:
            raise MemoryError("pinned ring allocation failed")
        self.nslots = nslots
        self.slot_bytes = int(self._lib.hds_ring_slot_bytes(self.h))
        self._views = []
        for i in range(nslots):
            p = self._lib.hds_ring_slot_ptr(self.h, i)
            arr = (ctypes.c_uint8 * self.slot_bytes).from_address(p)
            self._views.append(torch.frombuffer(arr, dtype=torch.uint8))

    def acquire(self):
        return self._lib.hds_ring_acquire(self.h)

    def slot(self, i, dtype=torch.uint8, numel=None):
        v = self._views[i]
        if dtype != torch.uint8:
            es = torch.tensor([], dtype=dtype).element_size()
            v = v[:(numel or self.slot_bytes // es) * es].view(dtype)
        elif numel is not None:
            v = v[:numel]
        return v

    def d2h(self, slot, dev_tensor, stream=None, offset=0):
        st = (stream or torch.cuda.current_stream()).cuda_stream
        native.check(self._lib.hds_ring_d2h(self.h, slot, dev_tensor.data_ptr(),
                                            dev_tensor.numel() * dev_tensor.element_size(), offset, st), "ring_d2h")

    def h2d(self, slot, dev_tensor, stream=None, offset=0):
        st = (stream or torch.cuda.current_stream()).cuda_stream
        native.check(self._lib.hds_ring_h2d(self.h, slot, dev_tensor.data_ptr(),
                                            dev_tensor.numel() * dev_tensor.element_size(), offset, st), "ring_h2d")

    def wait(self, slot):
        native.check(self._lib.hds_ring_wait(self.h, slot), "ring_wait")

    def stream_wait(self, slot, stream=None):
        st = (stream or torch.cuda.current_stream()).cuda_stream
        native.check(self._lib.hds_ring_stream_wait(self.h, slot, st), "ring_stream_wait")

    def done(self, slot):
        return bool(self._lib.hds_ring_query(self.h, slot))

    def __del__(self):
        try:
            if self.h:
                self._lib.hds_ring_destroy(self.h)
                self.h = None
        except Exception:
            pass


class PinnedPool:
    """Size-bucketed reuse pool of pinned host tensors (avoids hipHostMalloc on the training hot path)."""

    def __init__(self):
        self._free = {}
        self._lock = threading.Lock()
        self.bytes_allocated = 0

    @staticmethod
    def _bucket(nbytes):
        """Power-of-two buckets up to 64 MiB; above, 32 MiB granularity -- a 2.68 GB activation (Llama-3-8B block
        input at 320k tokens) would otherwise take a 4 GiB buffer, and 60 of them overran the host's memory budget."""
        n = int(nbytes)
        if n > (64 << 20):
            g = 32 << 20
            return (n + g - 1) // g * g
        return 1 << max(12, (n - 1).bit_length())

    @staticmethod
    def nbytes_of(t):
        """Pinned bytes behind a tensor from ``get`` (its bucket), or its own size."""
        buf = getattr(t, "_hds_pinned_owner", None)
        return buf.nbytes if buf is not None else t.numel() * t.element_size()

    def get(self, numel, dtype):
        es = torch.tensor([], dtype=dtype).element_size()
        b = self._bucket(numel * es)
        with self._lock:
            lst = self._free.get(b)
            buf = lst.pop() if lst else None
        if buf is None:
            buf = PinnedBuffer(b)
            self.bytes_allocated += b
        t = buf.view(dtype, numel)
        t._hds_pinned_owner = buf
        return t

    def get_tracked(self, numel, dtype):
        """Like ``get``, but the buffer goes back to the pool by itself once the returned tensor AND every view of
        it are gone."""
        import weakref
        es = torch.tensor([], dtype=dtype).element_size()
        b = self._bucket(numel * es)
        with self._lock:
            lst = self._free.get(b)
            buf = lst.pop() if lst else None
        if buf is None:
            buf = PinnedBuffer(b)
            self.bytes_allocated += b
        # the storage of a tensor made by from_numpy keeps that numpy array alive until the storage itself dies,
        # i.e. until the last tensor / view over it is gone: the finalizer rides on the array
        import numpy as np
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * buf.nbytes).from_address(buf.ptr))
        weakref.finalize(arr, self.put_buffer, buf)
        return torch.from_numpy(arr)[:numel * es].view(dtype)

    def put(self, t):
        buf = getattr(t, "_hds_pinned_owner", None)
        if buf is None:
            return
        self.put_buffer(buf)

    def put_buffer(self, buf):
        with self._lock:
            self._free.setdefault(buf.nbytes, []).append(buf)
