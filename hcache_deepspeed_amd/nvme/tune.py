"""``ds_nvme_tune``: sweep aio parameters and print the best ``aio`` config block (reference nvme/
perf_run_sweep.py + parse_nvme_stats.py, bin/ds_nvme_tune)."""
import argparse
import itertools
import json

from .ds_io import _parse_size, run_io


def sweep(folder, io_size="64M", block_sizes=("128K", "1M"), queue_depths=(8, 32), threads=(1, 4),
          single_submit=(False, ), overlap_events=(True, ), loops=2):
    results = []
    for rd in (True, False):
        for bs, qd, th, ss, oe in itertools.product(block_sizes, queue_depths, threads, single_submit,
                                                    overlap_events):
            results.append(run_io(folder, _parse_size(io_size), rd, _parse_size(bs), qd, th, ss, oe, loops))
    best = {}
    for op in ("read", "write"):
        rs = [r for r in results if r["op"] == op]
        best[op] = max(rs, key=lambda r: r["GB/s"]) if rs else None
    b = best["read"] or best["write"]
    aio = {"block_size": b["block_size"], "queue_depth": b["queue_depth"], "intra_op_parallelism":
           b["intra_op_parallelism"], "single_submit": b["single_submit"], "overlap_events": b["overlap_events"]}
    return results, best, {"aio": aio}


def main(argv=None):
    ap = argparse.ArgumentParser("ds_nvme_tune")
    ap.add_argument("--nvme_dir", required=True)
    ap.add_argument("--io_size", default="64M")
    ap.add_argument("--block_sizes", default="128K,1M")
    ap.add_argument("--queue_depths", default="8,32")
    ap.add_argument("--threads", default="1,4")
    a = ap.parse_args(argv)
    _, best, cfg = sweep(a.nvme_dir, a.io_size, a.block_sizes.split(","),
                         [int(x) for x in a.queue_depths.split(",")], [int(x) for x in a.threads.split(",")])
    for op, r in best.items():
        if r:
            print(f"best {op}: {r['GB/s']:.2f} GB/s  block={r['block_size']} qd={r['queue_depth']} "
                  f"threads={r['intra_op_parallelism']}")
    print(json.dumps(cfg, indent=2))
    return cfg


if __name__ == "__main__":
    main()
