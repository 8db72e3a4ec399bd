"""Which engine runs a side-stream host<->device copy, and what it costs the compute stream.

For each host buffer kind (torch pinned, hipHostMalloc portable) and direction, time: the copy alone, a GEMM loop
alone, and both concurrently (copy on a high-priority side stream). A copy executed by SDMA leaves the GEMMs at
their solo speed; one executed as a blit kernel (``__amd_rocclr_copyBuffer``, visible in a kernel trace) takes CUs
from them. Prints one JSON line per case plus the HIP/HSA environment.
"""
import json
import os
import sys
import time

sys.path.insert(0, ".")

import torch  # noqa: E402

from hcache_deepspeed_amd.offload.pinned import pinned_empty  # noqa: E402


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    env = {k: v for k, v in os.environ.items() if k.startswith(("HSA_", "HIP_", "GPU_", "ROC", "AMD_", "HCC_"))}
    print(json.dumps({"env": env}), flush=True)
    dev = torch.device("cuda")
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    n = (2 << 30) // 2  # 2 GiB bf16
    src = torch.randn(n, device=dev, dtype=torch.bfloat16)
    hosts = {"torch_pinned": torch.empty(n, dtype=torch.bfloat16, pin_memory=True),
             "hipHostMalloc": pinned_empty((n, ), torch.bfloat16)}
    side = torch.cuda.Stream(priority=-1)

    def gemms(k=40):
        for _ in range(k):
            torch.matmul(a, b)

    gemms(5)
    tg = wall(gemms)
    for name, h in hosts.items():
        for direction in ("d2h", "h2d"):
            def copy(reps=3):
                with torch.cuda.stream(side):
                    for _ in range(reps):
                        if direction == "d2h":
                            h.copy_(src, non_blocking=True)
                        else:
                            src.copy_(h, non_blocking=True)
            copy(1)
            tc = wall(copy)

            def both():
                copy()
                gemms()
            tb = wall(both)
            # GEMM time while the copy runs: launch both, time the GEMMs alone on the compute stream with events
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            copy()
            e0.record()
            gemms()
            e1.record()
            torch.cuda.synchronize()
            tge = e0.elapsed_time(e1)
            print(json.dumps({"host": name, "dir": direction, "copy_ms": round(tc, 1),
                              "copy_GBps": round(3 * 2 * n / tc / 1e6, 1), "gemm_alone_ms": round(tg, 1),
                              "gemm_with_copy_ms": round(tge, 1), "both_wall_ms": round(tb, 1),
                              "serial_sum_ms": round(tc + tg, 1)}), flush=True)


if __name__ == "__main__":
    main()
