"""NVMe-resident ZeRO-3 parameter shards (ZeRO-Infinity ``offload_param.device: nvme``).

Reference parity: runtime/swap_tensor/partitioned_param_swapper.py:37-422 (``AsyncPartitionedParameterSwapper``:
pinned swap buffers, ``swap_in`` / ``swap_out`` with async I/O, buffer_count x buffer_size).

This rank's compute-dtype shard of every unit lives in ``<folder>/params.swp`` in store order. A fetch reads a
unit's shard into one of ``buffer_count`` pinned staging buffers (the pool grows past that only when more
prefetches are in flight than buffers exist); the caller copies it H2D and releases the buffer. The optimizer
step writes updated shards back with async writes.
"""
import os

import torch

from .pipelined_optimizer_swapper import _pinned


class AsyncPartitionedParameterSwapper:

    def __init__(self, aio, folder, numel, dtype, buffer_numel, buffer_count=5):
        os.makedirs(folder, exist_ok=True)
        self.aio = aio
        self.file = os.path.join(folder, "params.swp")
        self.numel = int(numel)
        self.dtype = dtype
        self.esize = torch.tensor([], dtype=dtype).element_size()
        self.buffer_numel = int(max(1, buffer_numel))
        self.pool = [_pinned(self.buffer_numel, dtype) for _ in range(max(1, int(buffer_count)))]
        self.free = list(range(len(self.pool)))
        self.deferred = []  # (slot, device event): staging buffers whose H2D copy is still in flight
        self.bytes_read = self.bytes_written = 0
        with open(self.file, "ab"):
            pass

    # ---- staging buffers -------------------------------------------------------------------------
    def _acquire(self, n):
        assert n <= self.buffer_numel, f"swap request of {n} elements exceeds the {self.buffer_numel} buffer"
        if not self.free and self.deferred:
            still = []
            for slot, ev in self.deferred:
                if ev.query():
                    self.free.append(slot)
                else:
                    still.append((slot, ev))
            self.deferred = still
        if not self.free:
            self.pool.append(_pinned(self.buffer_numel, self.dtype))
            self.free.append(len(self.pool) - 1)
        return self.free.pop()

    def release(self, slot, event=None):
        """Return a staging buffer; with a device ``event`` it is reused only once that event has completed."""
        if event is None:
            self.free.append(slot)
        else:
            self.deferred.append((slot, event))

    # ---- transfers ---------------------------------------------------------------------------------
    def swap_in(self, lo, n):
        """Start reading elements [lo, lo + n) -> (slot, pinned view, AioRequest)."""
        slot = self._acquire(n)
        view = self.pool[slot][:n]
        req = self.aio.submit_read(view, self.file, lo * self.esize)
        self.bytes_read += n * self.esize
        return slot, view, req

    def swap_out(self, lo, src):
        """Start writing the pinned CPU tensor ``src`` to elements [lo, lo + numel)."""
        self.bytes_written += src.numel() * self.esize
        return self.aio.submit_write(src, self.file, lo * self.esize)

    def write_sync(self, lo, src):
        """Write any CPU/GPU tensor through a staging buffer (initialisation, checkpoint load)."""
        src = src.reshape(-1)
        for off in range(0, src.numel(), self.buffer_numel):
            n = min(self.buffer_numel, src.numel() - off)
            slot = self._acquire(n)
            buf = self.pool[slot][:n]
            buf.copy_(src[off:off + n])
            self.swap_out(lo + off, buf).wait()
            self.release(slot)

    def read_sync(self, lo, out):
        out = out.reshape(-1)
        for off in range(0, out.numel(), self.buffer_numel):
            n = min(self.buffer_numel, out.numel() - off)
            slot, view, req = self.swap_in(lo + off, n)
            req.wait()
            out[off:off + n].copy_(view)
            self.release(slot)
        return out
