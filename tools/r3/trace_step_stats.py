"""Per-kernel time and host<->device copy rates in the LAST training step of a rocprofv3 kernel + memory-copy trace
(the step window starts after the second-to-last optimizer kernel). Used to compare two builds' steps side by side.

    python tools/r3/trace_step_stats.py <rocprofv3 output dir>
"""
import collections
import csv
import glob
import os
import sys


def load(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main(d):
    ks = sorted(load(d, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    cs = load(d, "*memory_copy_trace.csv")
    if not ks:
        print("no kernel trace")
        return
    adam = [i for i, r in enumerate(ks) if "adam" in r["Kernel_Name"]]
    t0 = int(ks[adam[-2]]["End_Timestamp"]) if len(adam) >= 2 else int(ks[0]["Start_Timestamp"])
    t1 = int(ks[-1]["End_Timestamp"])
    print(f"step window {(t1 - t0) / 1e6:.1f} ms")
    agg = collections.defaultdict(lambda: [0, 0])
    for r in ks:
        a = int(r["Start_Timestamp"])
        if a < t0:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0][:90]
        agg[name][0] += 1
        agg[name][1] += int(r["End_Timestamp"]) - a
    tot = sum(v[1] for v in agg.values())
    print(f"kernel time {tot / 1e6:.1f} ms in {sum(v[0] for v in agg.values())} launches")
    for name, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"  {ns / 1e6:9.2f} ms {n:6d}x  {100 * ns / tot:5.1f}%  {name}")
    if cs:
        print("copy columns:", list(cs[0].keys()))
        by = collections.defaultdict(lambda: [0, 0, 0, None, None])
        for r in cs:
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if a < t0:
                continue
            k = r.get("Direction") or r.get("Kind") or r.get("Operation") or "?"
            nb = int(r.get("Size") or r.get("Bytes") or r.get("Copy_Bytes") or 0)
            v = by[k]
            v[0] += 1
            v[1] += nb
            v[2] += b - a
            v[3] = a if v[3] is None else min(v[3], a)
            v[4] = b if v[4] is None else max(v[4], b)
        for k, (n, nb, ns, a, b) in by.items():
            print(f"  {k}: {n} copies, {nb / 2**30:.1f} GiB, busy {ns / 1e6:.1f} ms "
                  f"({nb / max(ns, 1):.1f} GB/s while busy), span {(b - a) / 1e6:.1f} ms from step start "
                  f"+{(a - t0) / 1e6:.1f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
