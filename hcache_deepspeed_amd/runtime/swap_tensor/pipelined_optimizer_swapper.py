"""NVMe-resident fp32 master weights and optimizer moments, streamed through the optimizer step.

Reference parity: runtime/swap_tensor/partitioned_optimizer_swapper.py (one swap file per state) and
pipelined_optimizer_swapper.py:52-241 (overlap "read sub-group i+1 / update i / write i-1").

Each state of this rank's offloaded range lives in ``<folder>/<state>.swp`` (fp32, store order). The step walks
the range in chunks; :meth:`pipeline` yields chunk i's pinned staging views while the read of chunk i+1 and the
write-back of chunk i-1 are in flight on the async I/O engine (io_uring / thread pool, ops/aio.py). Three
staging slots per state make that overlap hazard-free: the read of chunk i+1 reuses the slot of chunk i-2,
whose write is awaited first.
"""
import os
import time

import torch

DEPTH = 3  # staging slots: read-ahead + in-use + write-behind


def _pinned(numel, dtype):
    if torch.cuda.is_available():
        from ...offload.pinned import pinned_empty
        return pinned_empty((int(numel), ), dtype)
    return torch.empty(int(numel), dtype=dtype)


class PipelinedOptimizerSwapper:

    def __init__(self, aio, folder, keys, numel, chunk_numel, dtype=torch.float32):
        os.makedirs(folder, exist_ok=True)
        self.aio = aio
        self.keys = list(keys)
        self.numel = int(numel)
        self.chunk = int(max(1, min(chunk_numel, max(1, numel))))
        self.dtype = dtype
        self.esize = torch.tensor([], dtype=dtype).element_size()
        self.files = {k: os.path.join(folder, f"{k}.swp") for k in self.keys}
        self.bufs = [{k: _pinned(self.chunk, dtype) for k in self.keys} for _ in range(DEPTH)]
        self.bytes_read = self.bytes_written = 0
        self.wait_s = 0.0  # time the step spent blocked on swap I/O (the rest overlapped the CPU update)
        self.step_s = 0.0  # wall time inside pipeline()

    # ---- whole-range transfers (init / checkpoint) ------------------------------------------------
    def write_full(self, key, src):
        """src: CPU tensor of ``numel`` elements (or None: zeros) -> the state's swap file, chunk by chunk."""
        buf = self.bufs[0][key]
        for lo in range(0, self.numel, self.chunk):
            n = min(self.chunk, self.numel - lo)
            if src is None:
                buf[:n].zero_()
            else:
                buf[:n].copy_(src[lo:lo + n])
            self.aio.submit_write(buf[:n], self.files[key], lo * self.esize).wait()
            self.bytes_written += n * self.esize

    def read_full(self, key, out=None):
        out = torch.empty(self.numel, dtype=self.dtype) if out is None else out
        buf = self.bufs[0][key]
        for lo in range(0, self.numel, self.chunk):
            n = min(self.chunk, self.numel - lo)
            self.aio.submit_read(buf[:n], self.files[key], lo * self.esize).wait()
            out[lo:lo + n].copy_(buf[:n])
            self.bytes_read += n * self.esize
        return out

    # ---- the pipelined step ---------------------------------------------------------------------------
    def pipeline(self, bounds):
        """bounds: [(lo, hi, ...)] with hi - lo <= chunk. Yields (i, {state: pinned view}) in order; the views are
        written back when the caller advances to the next chunk (or closes the generator)."""
        n = len(bounds)
        reads, writes = {}, {}

        def io(i, write):
            lo, hi = bounds[i][0], bounds[i][1]
            s = i % DEPTH
            sub = self.aio.submit_write if write else self.aio.submit_read
            nbytes = (hi - lo) * self.esize
            if write:
                self.bytes_written += nbytes * len(self.keys)
            else:
                self.bytes_read += nbytes * len(self.keys)
            return [sub(self.bufs[s][k][:hi - lo], self.files[k], lo * self.esize) for k in self.keys]

        def wait(reqs):
            t = time.perf_counter()
            for r in reqs:
                r.wait()
            self.wait_s += time.perf_counter() - t

        t0 = time.perf_counter()
        try:
            if n:
                reads[0] = io(0, False)
            for i in range(n):
                if i + 1 < n:
                    wait(writes.pop(i - 2, ()))  # slot of chunk i+1 == slot of chunk i-2
                    reads[i + 1] = io(i + 1, False)
                wait(reads.pop(i))
                lo, hi = bounds[i][0], bounds[i][1]
                s = i % DEPTH
                yield i, {k: self.bufs[s][k][:hi - lo] for k in self.keys}
                writes[i] = io(i, True)
        finally:
            for lst in list(reads.values()) + list(writes.values()):
                wait(lst)
            self.step_s += time.perf_counter() - t0
