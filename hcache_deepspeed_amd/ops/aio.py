"""Async tensor file I/O handle (reference: ``AsyncIOBuilder().load().aio_handle`` -- csrc/aio/py_lib/py_ds_aio.cpp
:19-115, and the GDS handle ``GDSBuilder().load().gds_handle``). Backed by csrc/host/aio.cpp (thread pool,
O_DIRECT for 4 KiB aligned pinned buffers).
"""
import os

import torch

from . import native


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
