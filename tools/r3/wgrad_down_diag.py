"""One weight-gradient layout at the Llama-3-8B down-projection shape (dY [T, 4096], X [T, 14336]), printing
before and after every GEMM so a stall names its call. Usage: wgrad_down_diag.py <layout> [N K]"""
import sys
import time

import torch

sys.path.insert(0, ".")


def main():
    from hcache_deepspeed_amd.ops import gemm
    lay = sys.argv[1]
    N, K = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (4096, 14336)
    T = 7 * 4096
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    ref = (dy.float().t() @ x.float())
    for i in range(4):
        t0 = time.perf_counter()
        print(f"{lay} call {i} start", flush=True)
        gemm._wgrad_run(lay, dy, x, out, False)
        torch.cuda.synchronize()
        print(f"{lay} call {i} done {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    print(f"{lay} rel err {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
