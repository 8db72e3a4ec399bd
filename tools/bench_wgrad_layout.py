"""Weight-gradient GEMM layouts at the bench shapes (T = 7 x 4096 tokens): dW[N,K] = dY[T,N]^T X[T,K].

  direct : torch.mm(dY.t(), X)                      (hipBLASLt TN, what autograd does)
  nt     : torch.mm(dYt, Xt.t()) on pre-transposed copies  (hipBLASLt NT: the fast forward layout)
  +tr    : nt plus the two transposes (torch copy)
"""
import sys
import time

import torch

sys.path.insert(0, ".")


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it


def main():
    T = 7 * 4096
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    tot = {"direct": 0.0, "nt+tr": 0.0}
    for name, (N, K) in shapes.items():
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * N * K
        td = t(lambda: torch.mm(dy.t(), x, out=out))
        dyt, xt = dy.t().contiguous(), x.t().contiguous()
        tn = t(lambda: torch.mm(dyt, xt.t(), out=out))
        from hcache_deepspeed_amd.ops.gemm import transpose2d
        ttr = t(lambda: (transpose2d(dy), transpose2d(x)))
        ref = torch.mm(dy.t(), x)
        err = (torch.mm(dyt, xt.t()).float() - ref.float()).abs().max().item()
        tot["direct"] += td
        tot["nt+tr"] += tn + ttr
        print(f"{name:8s} N={N:6d} K={K:6d}: direct {td*1e3:6.2f} ms ({fl/td/1e15:.2f} PF/s) | nt {tn*1e3:6.2f} ms "
              f"({fl/tn/1e15:.2f} PF/s) | HIP transposes {ttr*1e3:5.2f} ms ({(T*N+T*K)*4/ttr/1e12:.1f} TB/s) | "
              f"nt+tr {(tn+ttr)*1e3:6.2f} ms | maxdiff {err:.3g}", flush=True)
    print(f"per layer: direct {tot['direct']*1e3:.2f} ms, nt+transposes {tot['nt+tr']*1e3:.2f} ms")


def splitk():
    """Every wgrad candidate of ops/gemm.wgrad at the bench shapes (incl. two-stream split-K) + the auto pick."""
    from hcache_deepspeed_amd.ops import gemm
    T = 7 * 4096
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for name, (N, K) in shapes.items():
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * N * K
        res = {}
        ref = torch.mm(dy.t().float(), x.float())
        lays = ("direct", "nt", "direct_b2", "nt_b2") + (("direct_sk2", "nt_sk2") if "--streams" in sys.argv else ())
        for lay in lays:
            ts = t(lambda: gemm._wgrad_run(lay, dy, x, out, False))
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            res[lay] = (round(ts * 1e3, 3), round(fl / ts / 1e15, 3), round(err, 5))
        print(name, json.dumps(res), flush=True)


if __name__ == "__main__":
    import json
    splitk() if "--splitk" in sys.argv else main()
