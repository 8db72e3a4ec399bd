"""Which glue kernels run in the LAST training step of a rocprofv3 kernel trace, and between which kernels.

For every launch of a transpose / fill / D2D copy / dtype-copy kernel in the step window (after the second-to-last
optimizer kernel) prints its duration, grid and the names of the kernels around it; then totals per (kernel, grid).

    python tools/r3/glue_census.py <rocprofv3 output dir>
"""
import collections
import csv
import glob
import os
import sys

GLUE = ("transpose", "FillFunctor", "copyBuffer", "copy_kernel", "CUDAFunctor_add", "MulFunctor")


def short(n):
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    return n[:60]


def main(d):
    fs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    ks = sorted(csv.DictReader(open(fs[0])), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(ks) if "adam" in r["Kernel_Name"]]
    i0 = adam[-2] + 1 if len(adam) >= 2 else 0
    step = ks[i0:adam[-1] + 1] if adam else ks
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    print(f"step: {len(step)} launches, window {(t1 - t0) / 1e6:.1f} ms, kernel busy {busy / 1e6:.1f} ms")
    tot = collections.defaultdict(lambda: [0, 0])
    for j, r in enumerate(step):
        name = r["Kernel_Name"]
        if not any(g in name for g in GLUE):
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        grid = (r.get("Grid_Size_X") or r.get("Grid_Size", "?"), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))
        key = (short(name), grid)
        tot[key][0] += 1
        tot[key][1] += dur
        prev = short(step[j - 1]["Kernel_Name"]) if j else "-"
        nxt = short(step[j + 1]["Kernel_Name"]) if j + 1 < len(step) else "-"
        print(f"{j:5d} {dur / 1e3:8.1f} us  {short(name):40s} grid={grid}  after [{prev}]  before [{nxt}]")
    print("\ntotals per (kernel, grid):")
    for (n, g), (c, ns) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"  {ns / 1e6:8.2f} ms {c:5d}x  {n}  grid={g}")


if __name__ == "__main__":
    main(sys.argv[1])
