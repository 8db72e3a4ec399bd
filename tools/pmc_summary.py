"""MFMA utilisation per kernel of a training step from a rocprofv3 ``--pmc ... --kernel-trace`` run.

Reads ``*counter_collection.csv`` (per-dispatch counters) and ``*kernel_trace.csv`` (start/end), joins them on the
dispatch id and prints, per kernel name: calls, GPU time, achieved bf16 matrix FLOP/s from SQ_INSTS_VALU_MFMA_MOPS_BF16
(MOPS are counted in units of 512 FLOPs) against the 2.5 PF/s dense peak, and the MFMA-busy fraction
SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x SQ_BUSY_CU_CYCLES) when both were collected (per-SIMD MFMA-busy share of the
cycles the CUs were busy).

Usage: python tools/pmc_summary.py <rocprof output dir> [out.csv]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

PEAK = 2.5e15


def _read(pattern):
    fs = glob.glob(pattern, recursive=True)
    rows = []
    for f in fs:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main(d, out=None):
    ctr = _read(os.path.join(d, "**", "*counter_collection.csv"))
    trace = _read(os.path.join(d, "**", "*kernel_trace.csv"))
    dur = {}
    for r in trace:
        dur[r.get("Dispatch_Id")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"])
    per = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    for r in ctr:
        did = r.get("Dispatch_Id")
        name = r.get("Kernel_Name") or dur.get(did, (0, "?"))[1]
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        if did not in seen[name]:
            seen[name].add(did)
            per[name]["_ns"] += dur.get(did, (0, ""))[0]
            per[name]["_calls"] += 1
    rows = []
    for name, c in per.items():
        ns = c["_ns"]
        flops = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        cu = c.get("SQ_BUSY_CU_CYCLES")
        rows.append((name, int(c["_calls"]), ns / 1e6, flops / (ns * 1e-9) if ns else 0.0,
                     (busy / (4 * cu)) if busy and cu else None))
    rows.sort(key=lambda r: -r[2])
    tot_ms = sum(r[2] for r in rows)
    tot_fl = sum(r[3] * r[2] * 1e-3 for r in rows)
    lines = [f"{'ms':>9} {'calls':>6} {'PF/s':>6} {'of peak':>7} {'mfma busy':>9}  kernel"]
    for name, n, ms, fs, b in rows[:40]:
        lines.append(f"{ms:9.2f} {n:6d} {fs / 1e15:6.3f} {100 * fs / PEAK:6.1f}% "
                     f"{'' if b is None else f'{100 * b:8.1f}%'}  {name[:100]}")
    lines.append(f"total {tot_ms:.1f} ms of kernels, {tot_fl / 1e12:.1f} TFLOP on MFMA "
                 f"-> {tot_fl / (tot_ms * 1e-3) / 1e15:.3f} PF/s averaged over kernel time")
    print("\n".join(lines))
    if out:
        with open(out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
