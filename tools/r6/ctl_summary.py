"""One line per host-activation-cache control run: tok/s, timed-step peak, spilled bytes, recomputed blocks, measured
resident-block footprint, per-step peaks (tools/r6/gpu_controls.sh)."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
a = d["extra"].get("act_cache", {})
print(sys.argv[2], d["value"], d["extra"].get("peak_gib_timed_steps"), a.get("bytes_offloaded"),
      a.get("recomputed_layers"), a.get("resident_block_gib"), a.get("step_peaks_gib"))
