"""Host<->device copy bandwidth through the framework's pinned buffers (hipHostMalloc) vs torch pin_memory.

    python tools/pcie_bw.py [--gib 4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4)
    a = ap.parse_args()
    import torch
    from hcache_deepspeed_amd.offload.pinned import pinned_empty
    n = int(a.gib * 2**30)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    res = {}
    for name, host in (("hipHostMalloc", pinned_empty((n, ), torch.uint8)),
                       ("torch_pin_memory", torch.empty(n, dtype=torch.uint8).pin_memory())):
        s = torch.cuda.Stream()
        for direction in ("d2h", "h2d"):
            for _ in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                with torch.cuda.stream(s):
                    (host.copy_(dev, non_blocking=True) if direction == "d2h" else dev.copy_(host, non_blocking=True))
                s.synchronize()
                dt = time.perf_counter() - t0
            res[f"{name}_{direction}_GBps"] = round(n / dt / 1e9, 1)
        # both directions at once on two streams
        s2 = torch.cuda.Stream()
        dev2 = torch.empty_like(dev)
        host2 = pinned_empty((n, ), torch.uint8)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            host.copy_(dev, non_blocking=True)
        with torch.cuda.stream(s2):
            dev2.copy_(host2, non_blocking=True)
        torch.cuda.synchronize()
        res[f"{name}_bidir_GBps"] = round(2 * n / (time.perf_counter() - t0) / 1e9, 1)
        del host
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
