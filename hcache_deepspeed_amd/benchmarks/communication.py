"""``ds_bench``: collective bandwidth benchmark over RCCL (xGMI) or gloo.

Reference parity: bin/ds_bench (imports ``benchmarks.communication`` from DeepSpeedExamples, not shipped with the
reference) -- all_reduce / all_gather / reduce_scatter / all_to_all / broadcast / pt2pt sweeps reporting latency,
algbw and busbw with the nccl-tests formulas (utils/comms_logging.calc_bw: all-reduce 2(n-1)/n, AG/RS (n-1)/n).

On an 8x MI355X node this is the tool for sizing ZeRO bucket sizes to the 7 point-to-point xGMI links: run
``python -m torch.distributed.run --nproc-per-node 8 -m hcache_deepspeed_amd.benchmarks.communication --scan``.
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as tdist

from ..utils.comms_logging import calc_bw

OPS = ("all_reduce", "all_gather", "reduce_scatter", "all_to_all", "broadcast", "pt2pt")


def _run_op(op, n_elems, dtype, device, world, rank):
    es = torch.tensor([], dtype=dtype).element_size()
    if op == "all_reduce":
        t = torch.ones(n_elems, dtype=dtype, device=device)
        return (lambda: tdist.all_reduce(t)), n_elems * es
    if op == "all_gather":
        per = max(1, n_elems // world)
        src = torch.ones(per, dtype=dtype, device=device)
        out = torch.empty(per * world, dtype=dtype, device=device)
        return (lambda: tdist.all_gather_into_tensor(out, src)), per * world * es
    if op == "reduce_scatter":
        per = max(1, n_elems // world)
        src = torch.ones(per * world, dtype=dtype, device=device)
        out = torch.empty(per, dtype=dtype, device=device)
        return (lambda: tdist.reduce_scatter_tensor(out, src)), per * world * es
    if op == "all_to_all":
        per = max(1, n_elems // world) * world
        src = torch.ones(per, dtype=dtype, device=device)
        out = torch.empty(per, dtype=dtype, device=device)
        return (lambda: tdist.all_to_all_single(out, src)), per * es
    if op == "broadcast":
        t = torch.ones(n_elems, dtype=dtype, device=device)
        return (lambda: tdist.broadcast(t, 0)), n_elems * es
    if op == "pt2pt":
        t = torch.ones(n_elems, dtype=dtype, device=device)
        peer = rank ^ 1

        def f():
            if peer >= world:
                return
            if rank % 2 == 0:
                tdist.send(t, peer)
                tdist.recv(t, peer)
            else:
                tdist.recv(t, peer)
                tdist.send(t, peer)

        return f, n_elems * es
    raise ValueError(op)


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def bench(ops=OPS, sizes=(1 << 20, ), dtype=torch.bfloat16, trials=10, warmups=3, device=None):
    """Returns a list of result dicts (rank-0 max latency over ranks)."""
    world, rank = tdist.get_world_size(), tdist.get_rank()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if tdist.get_backend() == "nccl" \
            else torch.device("cpu")
    results = []
    for op in ops:
        for nbytes in sizes:
            n = max(world, nbytes // torch.tensor([], dtype=dtype).element_size())
            fn, size = _run_op(op, n, dtype, device, world, rank)
            for _ in range(warmups):
                fn()
            _sync(device)
            tdist.barrier()
            t0 = time.perf_counter()
            for _ in range(trials):
                fn()
            _sync(device)
            lat = torch.tensor([(time.perf_counter() - t0) / trials * 1e3], dtype=torch.float64)
            tdist.all_reduce(lat, op=tdist.ReduceOp.MAX)
            lat_ms = float(lat.item())
            name = {"pt2pt": "send", "all_to_all": "all_to_all_single", "all_gather": "all_gather_into_tensor",
                    "reduce_scatter": "reduce_scatter_tensor"}.get(op, op)
            algbw, busbw = (x / 8 for x in calc_bw(name, size, lat_ms, world))  # Gbit/s -> GB/s
            results.append({"op": op, "bytes": size, "lat_ms": round(lat_ms, 4), "algbw_GBps": round(algbw, 3),
                            "busbw_GBps": round(busbw, 3), "world": world, "dtype": str(dtype).split(".")[-1]})
    return results


def main(argv=None):
    ap = argparse.ArgumentParser("ds_bench")
    ap.add_argument("--ops", default=",".join(OPS))
    ap.add_argument("--scan", action="store_true", help="sweep 64 KiB .. 1 GiB")
    ap.add_argument("--maxsize", type=int, default=24, help="log2 bytes of the single size when not scanning")
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--warmups", type=int, default=3)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--backend", default=None)
    a = ap.parse_args(argv)
    if not tdist.is_initialized():
        backend = a.backend or ("nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29555")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        tdist.init_process_group(backend)
    sizes = [1 << p for p in range(16, 31, 2)] if a.scan else [1 << a.maxsize]
    res = bench(a.ops.split(","), sizes, getattr(torch, a.dtype), a.trials, a.warmups)
    if tdist.get_rank() == 0:
        for r in res:
            print(json.dumps(r), flush=True)
    return res


if __name__ == "__main__":
    main()
