"""Fused Adam (hds_adam_flat) at ZeRO-3 dp1 Llama-3-8B-like size: fp32 master/m/v, bf16 grad, bf16 copy.
Prints ms and effective TB/s (28 B moved per element). Run once per HDS_ADAM_NT setting (read once per process)."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops import native  # noqa: E402


def main():
    n = int(os.environ.get("ADAM_N", str(2_000_000_000)))
    lib = native.kernels()
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    lp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    st = native.stream()
    call = lambda: lib.hds_adam_flat(native.dt(p), native.dt(g), p.data_ptr(), g.data_ptr(), m.data_ptr(),  # noqa
                                     v.data_ptr(), lp.data_ptr(), n, 1e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.05, 1, 1.0,
                                     None, None, st)
    for _ in range(3):
        assert call() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    e0.record()
    for _ in range(it):
        call()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(json.dumps({"n": n, "nt": os.environ.get("HDS_ADAM_NT", "0"), "ms": round(ms, 3),
                      "TBps": round(28 * n / ms / 1e9, 2), "ms_at_8.03B": round(ms * 8.03e9 / n, 2)}), flush=True)


if __name__ == "__main__":
    main()
