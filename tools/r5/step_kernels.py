"""Per-kernel time of the LAST training step in a rocprofv3 database (kernels view): the step is the window between
the last two fused-Adam dispatches (one per step). Usage: python tools/r5/step_kernels.py run_results.db [out.txt]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
adam = [r for r in rows if "adam_flat" in r[0]]
# one optimizer step may launch several fused-Adam kernels (e.g. dense + expert parameter groups): dispatches closer
# than 50 ms apart belong to the same step, whose end is its last dispatch
ends = []
for r in adam:
    if ends and r[1] - ends[-1] < 50e6:
        ends[-1] = r[2]
    else:
        ends.append(r[2])
if len(ends) < 2:
    raise SystemExit("fewer than two optimizer steps in the trace")
t0, t1 = ends[-2], ends[-1]
tot = defaultdict(float)
cnt = defaultdict(int)
for n, s, e in rows:
    if s >= t0 and e <= t1:
        tot[n] += (e - s) / 1e6
        cnt[n] += 1
busy = sum(tot.values())
lines = [f"# last step of the traced run (window between the last two fused-Adam dispatches)",
         f"step window {(t1 - t0) / 1e6:.1f} ms", f"kernel time {busy:.1f} ms in {sum(cnt.values())} launches"]
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:30]:
    lines.append(f"{t:10.2f} ms {cnt[n]:6d}x {100 * t / busy:6.1f}%  {n[:110]}")
out = "\n".join(lines)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
