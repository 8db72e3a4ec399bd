# v2 serving decode at B=1 (Llama-3-8B, 512-token prompt): throughput, then a kernel trace of the same run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6dec${B:-1}
mkdir -p $O
timeout -k 10 300 python tools/bench_v2_decode.py --batches ${B:-1} --steps 64 > $O/decode_b${B:-1}.jsonl 2> $O/decode_b${B:-1}.err || { echo failed; tail -20 $O/decode_b${B:-1}.err; exit 1; }
cat $O/decode_b${B:-1}.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/bench_v2_decode.py --batches ${B:-1} --steps 64 > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
DB=$(find $O/prof -name "*.db" | head -1)
python - "$DB" <<'PY' > $O/decode_kernels.txt
import sqlite3, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
# the last 64 decode steps: from the 64th-to-last lm-head-sized GEMV... simply the last 40 % of the trace
t_end = rows[-1][2]; t0 = rows[int(len(rows) * 0.6)][1]
tot = defaultdict(float); cnt = defaultdict(int)
for n, s, e in rows:
    if s >= t0:
        tot[n] += (e - s) / 1e6; cnt[n] += 1
busy = sum(tot.values())
print(f"window {(t_end - t0) / 1e6:.1f} ms, kernel time {busy:.1f} ms, {sum(cnt.values())} launches")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:25]:
    print(f"{t:9.2f} ms {cnt[n]:6d}x {100 * t / busy:5.1f}%  {n[:100]}")
PY
cat $O/decode_kernels.txt | head -20
find $O/prof -name "*.db" -size +30M -delete
