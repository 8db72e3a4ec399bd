"""Summarise a rocprofv3 rocpd SQLite database into per-kernel stats CSV (name, calls, total_ms, avg_us, pct).

Usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db profiles/out.csv [--steps N]
"""
import csv
import sqlite3
import sys


def main(db, out, steps=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start) from kernels group by name "
                     "order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ms", "avg_us", "pct"] + (["ms_per_step"] if steps else []))
        for name, n, ns in rows:
            extra = [f"{ns / 1e6 / steps:.3f}"] if steps else []
            w.writerow([name[:160], n, f"{ns / 1e6:.3f}", f"{ns / 1e3 / n:.2f}", f"{100 * ns / total:.2f}"] + extra)
    print(f"{len(rows)} kernels, total GPU kernel time {total / 1e6:.1f} ms")


if __name__ == "__main__":
    a = sys.argv[1:]
    steps = None
    if "--steps" in a:
        i = a.index("--steps")
        steps = int(a[i + 1])
        del a[i:i + 2]
    main(a[0], a[1], steps)
