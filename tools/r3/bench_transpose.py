"""HIP bf16 transpose variants at the step's shapes (T = 7 x 4096 tokens): GB/s of read + write."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")


def main():
    from hcache_deepspeed_amd.ops.gemm import transpose2d
    T = 7 * 4096
    for name, (R, C) in {"act_4096": (T, 4096), "dy_gate_up": (T, 28672), "dl_lm_chunk": (4096, 128256),
                         "w_gate_up": (28672, 4096), "w_lm": (128256, 4096), "w_qkv": (6144, 4096)}.items():
        x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
        res = {}
        for var in (1, 2):
            y = transpose2d(x, variant=var)
            torch.cuda.synchronize()
            it = 20
            t0 = time.perf_counter()
            for _ in range(it):
                y = transpose2d(x, variant=var)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / it
            ok = torch.equal(y, x.t().contiguous())
            res[var] = {"us": round(dt * 1e6, 1), "TBps": round(4 * R * C / dt / 1e12, 2), "ok": ok}
        print(json.dumps({"shape": name, "R": R, "C": C, **{f"v{k}": v for k, v in res.items()}}), flush=True)
        del x, y


if __name__ == "__main__":
    main()
