"""Multi-process test harness (reference: tests/unit/common.py DistributedExec/DistributedTest :129-493).

``run_distributed(fn, world_size, *args)`` spawns ``world_size`` processes, rendezvous through a file
store in a temp dir (no network / hostname resolution), backend gloo on CPU, and re-raises the first
failure in the parent. ``fn(rank, world_size, *args)`` runs with torch.distributed initialised.
"""
import os
import tempfile
import traceback

import torch.multiprocessing as mp


def _worker(rank, world_size, fn, args, init_file, err_q, backend):
    try:
        os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world_size), LOCAL_SIZE=str(world_size),
                          MASTER_ADDR="127.0.0.1")
        os.environ.setdefault("OMP_NUM_THREADS", "2")
        import torch
        import torch.distributed as dist
        torch.set_num_threads(2)
        dist.init_process_group(backend, init_method=f"file://{init_file}", rank=rank, world_size=world_size)
        from hcache_deepspeed_amd.utils import groups
        groups.reset()
        fn(rank, world_size, *args)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:  # noqa: B902
        err_q.put((rank, traceback.format_exc()))
        raise


def run_distributed(fn, world_size=2, *args, backend="gloo", timeout=600):
    ctx = mp.get_context("spawn")
    err_q = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        init_file = os.path.join(d, "store")
        procs = [ctx.Process(target=_worker, args=(r, world_size, fn, args, init_file, err_q, backend))
                 for r in range(world_size)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout)
        for p in procs:
            if p.is_alive():
                p.kill()
                raise TimeoutError("distributed test timed out")
        if not err_q.empty():
            rank, tb = err_q.get()
            raise AssertionError(f"rank {rank} failed:\n{tb}")
        for p in procs:
            assert p.exitcode == 0, f"process exit code {p.exitcode}"
