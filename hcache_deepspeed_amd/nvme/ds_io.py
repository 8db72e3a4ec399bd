"""``ds_io``: read / write throughput of the async file tier (reference nvme/ds_aio_handle.py :22-222, bin/ds_io).

Each process moves ``--io_size`` bytes between a pinned host buffer (optionally a GPU tensor staged through it,
``--gpu``) and ``--folder``/``<rank>.bin`` with the C++ aio handle (csrc/host/aio.cpp: thread pool, O_DIRECT
for 4 KiB-aligned pinned buffers), ``--loops`` times, and reports GB/s.
"""
import argparse
import json
import os
import time

import torch


def _parse_size(s):
    s = str(s).strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * mult[s[-1]]) if s[-1] in mult else int(s)


def run_io(folder, io_size, read=True, block_size=1 << 20, queue_depth=32, intra_op_parallelism=4,
           single_submit=False, overlap_events=True, loops=3, gpu=False, rank=0):
    from ..offload.pinned import pinned_empty
    from ..ops.aio import aio_handle
    os.makedirs(folder, exist_ok=True)
    path = os.path.join(folder, f"ds_io_{rank}.bin")
    n = (io_size + 4095) // 4096 * 4096
    # pinned (hipHostMalloc) buffer on a GPU machine; plain host memory (buffered I/O) without a GPU runtime
    buf = pinned_empty((n, ), torch.uint8) if torch.cuda.is_available() else torch.empty(n, dtype=torch.uint8)
    h = aio_handle(block_size, queue_depth, single_submit, overlap_events, intra_op_parallelism)
    if read and (not os.path.exists(path) or os.path.getsize(path) < n):
        buf.fill_(7)
        h.sync_pwrite(buf, path)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda") if gpu and torch.cuda.is_available() else None
    times = []
    for _ in range(loops):
        if not read and dev is not None:
            buf.copy_(dev, non_blocking=False)
        t0 = time.perf_counter()
        if read:
            h.async_pread(buf, path)
        else:
            h.async_pwrite(buf, path)
        h.wait()
        if read and dev is not None:
            dev.copy_(buf, non_blocking=True)
            torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    best = min(times)
    return {"op": "read" if read else "write", "bytes": n, "best_s": best, "GB/s": n / best / 1e9,
            "block_size": block_size, "queue_depth": queue_depth, "intra_op_parallelism": intra_op_parallelism,
            "single_submit": single_submit, "overlap_events": overlap_events, "gpu": bool(dev is not None)}


def main(argv=None):
    ap = argparse.ArgumentParser("ds_io")
    ap.add_argument("--folder", required=True)
    ap.add_argument("--io_size", default="64M")
    ap.add_argument("--read", action="store_true")
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--block_size", default="1M")
    ap.add_argument("--queue_depth", type=int, default=32)
    ap.add_argument("--threads", "--intra_op_parallelism", dest="threads", type=int, default=4)
    ap.add_argument("--single_submit", action="store_true")
    ap.add_argument("--sequential_requests", action="store_true", help="disable overlap_events")
    ap.add_argument("--loops", type=int, default=3)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args(argv)
    ops = ([True] if a.read or not a.write else []) + ([False] if a.write else [])
    out = []
    for rd in ops:
        r = run_io(a.folder, _parse_size(a.io_size), rd, _parse_size(a.block_size), a.queue_depth, a.threads,
                   a.single_submit, not a.sequential_requests, a.loops, a.gpu)
        print(json.dumps(r))
        out.append(r)
    return out


if __name__ == "__main__":
    main()
