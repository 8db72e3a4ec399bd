"""Async tensor file I/O handle (reference: ``AsyncIOBuilder().load().aio_handle`` -- csrc/aio/py_lib/py_ds_aio.cpp
:19-115, and the GDS handle ``GDSBuilder().load().gds_handle``). Backed by csrc/host/aio.cpp: io_uring (raw
syscalls, block_size chunks, queue_depth in flight) or a pread/pwrite thread pool; O_DIRECT for 4 KiB aligned
pinned buffers. Beyond the reference API, :meth:`aio_handle.submit_read` / :meth:`aio_handle.submit_write` return an
:class:`AioRequest` whose ``wait()`` blocks on that request only (what a read-ahead / write-behind pipeline needs).
"""
import os

import torch

from . import native


class AioRequest:
    """One in-flight tracked transfer; keeps its buffer alive until waited."""

    __slots__ = ("handle", "rid", "buffer", "done")

    def __init__(self, handle, rid, buffer):
        self.handle, self.rid, self.buffer, self.done = handle, rid, buffer, False

    def wait(self):
        if not self.done:
            rc = self.handle._lib.hds_aio_wait_req(self.handle.h, self.rid)
            self.done = True
            self.buffer = None
            if rc != 0:
                raise IOError(f"aio request {self.rid} failed ({rc})")
        return True


class aio_handle:

    def __init__(self, block_size=1 << 20, queue_depth=128, single_submit=False, overlap_events=True,
                 intra_op_parallelism=4):
        self._lib = native.host_lib()
        self.h = self._lib.hds_aio_create(int(block_size), int(queue_depth), int(single_submit), int(overlap_events),
                                          int(intra_op_parallelism))
        self.block_size, self.queue_depth = block_size, queue_depth
        self.single_submit, self.overlap_events = single_submit, overlap_events
        self.intra_op_parallelism = intra_op_parallelism
        self._pool_refs = []

    # reference getters
    def get_block_size(self):
        return self.block_size

    def get_queue_depth(self):
        return self.queue_depth

    def get_single_submit(self):
        return self.single_submit

    def get_overlap_events(self):
        return self.overlap_events

    def get_intra_op_parallelism(self):
        return self.intra_op_parallelism

    @property
    def engine(self):
        """"io_uring" or "threads"."""
        return "io_uring" if self._lib.hds_aio_engine(self.h) == 1 else "threads"

    def _submit(self, write, buffer, filename, file_offset):
        p, n = self._buf(buffer)
        rid = self._lib.hds_aio_submit(self.h, int(write), p, n, filename.encode(), int(file_offset))
        if rid <= 0:
            raise IOError(f"aio {'write' if write else 'read'} of {filename} failed to submit ({rid})")
        return AioRequest(self, rid, buffer)

    def submit_read(self, buffer, filename, file_offset=0):
        return self._submit(False, buffer, filename, file_offset)

    def submit_write(self, buffer, filename, file_offset=0):
        return self._submit(True, buffer, filename, file_offset)

    def _buf(self, t):
        assert not t.is_cuda, "aio buffers must be host tensors (pinned preferred)"
        assert t.is_contiguous()
        return t.data_ptr(), t.numel() * t.element_size()

    def pread(self, buffer, filename, validate=False, async_op=False, file_offset=0):
        p, n = self._buf(buffer)
        if self._lib.hds_aio_pread(self.h, p, n, filename.encode(), int(file_offset), int(async_op)) != 0:
            raise IOError(f"aio read of {filename} failed")
        return 1

    def pwrite(self, buffer, filename, validate=False, async_op=False, file_offset=0):
        p, n = self._buf(buffer)
        if self._lib.hds_aio_pwrite(self.h, p, n, filename.encode(), int(file_offset), int(async_op)) != 0:
            raise IOError(f"aio write of {filename} failed")
        return 1

    def sync_pread(self, buffer, filename, file_offset=0):
        return self.pread(buffer, filename, async_op=False, file_offset=file_offset)

    def sync_pwrite(self, buffer, filename, file_offset=0):
        return self.pwrite(buffer, filename, async_op=False, file_offset=file_offset)

    def async_pread(self, buffer, filename, file_offset=0):
        return self.pread(buffer, filename, async_op=True, file_offset=file_offset)

    def async_pwrite(self, buffer, filename, file_offset=0):
        return self.pwrite(buffer, filename, async_op=True, file_offset=file_offset)

    read = sync_pread
    write = sync_pwrite

    def wait(self):
        n = self._lib.hds_aio_wait(self.h)
        if n < 0:
            raise IOError(f"{-n} aio chunk(s) failed")
        return n

    def new_cpu_locked_tensor(self, num_elem, example_tensor):
        from ..offload.pinned import pinned_empty
        t = pinned_empty((int(num_elem), ), example_tensor.dtype)
        self._pool_refs.append(t)
        return t

    def free_cpu_locked_tensor(self, tensor):
        self._pool_refs = [t for t in self._pool_refs if t.data_ptr() != tensor.data_ptr()]
        return True

    def __del__(self):
        try:
            if self.h:
                self._lib.hds_aio_destroy(self.h)
                self.h = None
        except Exception:
            pass


# the GPUDirect-Storage handle has the same API; on MI355X it bounces through pinned host memory
gds_handle = aio_handle


class AsyncIOBuilder:
    """``AsyncIOBuilder().load()`` compatibility shim returning this module."""

    NAME = "async_io"

    def is_compatible(self, verbose=False):
        return True

    def load(self, verbose=False):
        import sys
        return sys.modules[__name__]


def file_size(path):
    return native.host_lib().hds_aio_file_size(path.encode())
