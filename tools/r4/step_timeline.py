"""Timeline of the LAST training step in a rocprofv3 kernel (+ memory-copy) trace: GPU busy fraction, the longest
idle gaps (when, how long, what ran before and after), the forward / backward split (at the cross-entropy kernels),
and per direction how many bytes the host<->device copies moved in each phase and how busy the copy engine was.

    python tools/r4/step_timeline.py <rocprofv3 output dir> [--gaps 12]
"""
import argparse
import collections
import csv
import glob
import os


def load(d, pat):
    fs = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
    rows = []
    for f in fs:
        rows += list(csv.DictReader(open(f)))
    return rows


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    ks = sorted(load(a.dir, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    cs = load(a.dir, "*memory_copy_trace.csv")
    if not ks:
        print("no kernel trace")
        return
    opt = [i for i, r in enumerate(ks) if "adam" in r["Kernel_Name"]]
    t0 = int(ks[opt[-2]]["End_Timestamp"]) if len(opt) >= 2 else int(ks[0]["Start_Timestamp"])
    t1 = int(ks[opt[-1]]["End_Timestamp"]) if opt else int(ks[-1]["End_Timestamp"])
    step = [r for r in ks if t0 <= int(r["Start_Timestamp"]) < t1]
    iv = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step])
    busy = sum(b - x for x, b in iv)
    span = t1 - t0
    xent = [int(r["Start_Timestamp"]) for r in step if "xent" in r["Kernel_Name"]]
    turn = min(xent) if xent else None
    print(f"step window {span / 1e6:.1f} ms, GPU busy {100 * busy / span:.2f} %, idle {(span - busy) / 1e6:.1f} ms"
          + (f", forward {(turn - t0) / 1e6:.1f} ms / rest {(t1 - turn) / 1e6:.1f} ms" if turn else ""))
    gaps = []
    prev_end, prev_name = t0, "(step start)"
    starts = {(int(r["Start_Timestamp"])): r["Kernel_Name"].split("(")[0][:60] for r in step}
    for x, b in iv:
        if x > prev_end:
            gaps.append((x - prev_end, prev_end, prev_name, starts.get(x, "?")))
        prev_end = b
        prev_name = next((r["Kernel_Name"].split("(")[0][:60] for r in step if int(r["End_Timestamp"]) == b), "?")
    gaps.sort(reverse=True)
    print(f"longest gaps (of {len(gaps)}):")
    for g, at, before, after in gaps[:a.gaps]:
        ph = "" if turn is None else (" fwd" if at < turn else " bwd")
        print(f"  {g / 1e6:8.2f} ms at +{(at - t0) / 1e6:8.1f} ms{ph}  after {before}  before {after}")
    if not cs:
        return
    by = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0, 0]))
    for r in cs:
        x, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if not (t0 <= x < t1):
            continue
        k = r.get("Direction") or r.get("Kind") or r.get("Operation") or "?"
        nb = int(r.get("Size") or r.get("Bytes") or r.get("Copy_Bytes") or 0)
        ph = "all" if turn is None else ("fwd" if x < turn else "bwd")
        v = by[k][ph]
        v[0] += 1
        v[1] += nb
        v[2] += b - x
    for k, phases in by.items():
        for ph, (n, nb, ns) in sorted(phases.items()):
            print(f"  {k:>22s} {ph}: {n:5d} copies {nb / 2**30:7.2f} GiB busy {ns / 1e6:8.1f} ms "
                  f"({nb / max(ns, 1):5.1f} GB/s while busy)")


if __name__ == "__main__":
    main()
