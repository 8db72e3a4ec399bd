"""Summarise a rocprofv3 kernel + memory-copy trace of one training step: how much of the host<->device copy
time overlaps kernel execution, and the longest stretches where copies ran with no kernel (compute waiting)."""
import csv
import glob
import os
import sys


def load(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main(d):
    ks = load(d, "*kernel_trace.csv")
    cs = load(d, "*memory_copy_trace.csv")
    if not ks or not cs:
        print("missing traces", len(ks), len(cs))
        return
    kiv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks)
    # the last step: after the last optimizer kernel of the warmup ... use the last 45% of the kernel timeline
    t_end = kiv[-1][1]
    adam = [i for i, r in enumerate(sorted(ks, key=lambda r: int(r["Start_Timestamp"]))) if "adam" in r["Kernel_Name"]]
    ks_sorted = sorted(ks, key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(ks_sorted[adam[-2]]["End_Timestamp"]) if len(adam) >= 2 else kiv[0][0]
    kiv = [(a, b) for a, b in kiv if a >= t0]
    civ = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Kind", "")))
                 for r in cs if int(r["Start_Timestamp"]) >= t0)
    # merge kernel busy intervals
    busy = []
    for a, b in kiv:
        if busy and a <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], b)
        else:
            busy.append([a, b])

    def overlap(a, b):
        tot = 0
        for x, y in busy:
            if y <= a:
                continue
            if x >= b:
                break
            tot += min(b, y) - max(a, x)
        return tot

    copy_ns = sum(b - a for a, b, _ in civ)
    ov = sum(overlap(a, b) for a, b, _ in civ)
    gaps = []
    for (a1, b1), (a2, b2) in zip(busy, busy[1:]):
        if a2 - b1 > 0:
            gaps.append(a2 - b1)
    gaps.sort(reverse=True)
    step = kiv[-1][1] - t0
    nbytes = sum(int(r.get("Size", r.get("Bytes", 0)) or 0) for r in cs if int(r["Start_Timestamp"]) >= t0)
    print(f"step window {step/1e6:.1f} ms, kernel busy {sum(b-a for a,b in busy)/1e6:.1f} ms, copies {len(civ)} "
          f"({nbytes/2**30:.1f} GiB) taking {copy_ns/1e6:.1f} ms, {100*ov/max(1,copy_ns):.1f}% of copy time "
          f"overlapped by kernels")
    print("longest kernel-idle gaps (ms):", [round(g / 1e6, 2) for g in gaps[:10]])
    print("idle gaps > 1 ms:", sum(1 for g in gaps if g > 1e6), "total idle ms:", round(sum(gaps) / 1e6, 1))


if __name__ == "__main__":
    main(sys.argv[1])
