"""GEMM microbenchmark: hand-written MFMA kernel (ops/gemm.py) vs torch.matmul (hipBLASLt) at the Llama-3-8B
projection shapes of the bench (M = 7 x 4096 tokens). Random N(0,1) bf16 data; interleaved rounds in one
process; prints one JSON line per shape."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.fp8_gemm import mx_gemm, mx_quantize  # noqa: E402
from hcache_deepspeed_amd.ops.gemm import gemm_nt  # noqa: E402

SHAPES = [  # (M, N, K, name)
    (28672, 6144, 4096, "qkv"),
    (28672, 4096, 4096, "o_proj"),
    (28672, 28672, 4096, "gate_up"),
    (28672, 4096, 14336, "down"),
]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    torch.manual_seed(0)
    # correctness on a small asymmetric case against an fp32 reference
    a = torch.randn(512, 384, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(768, 384, device="cuda", dtype=torch.bfloat16)
    ref = a.float() @ b.float().t()
    got = gemm_nt(a, b).float()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps({"check": "512x768x384", "max_rel_err": err}), flush=True)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for M, N, K, name in SHAPES:
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        qa, sa = mx_quantize(a)
        qb, sb = mx_quantize(b)
        fns = {"v0": lambda: gemm_nt(a, b, out=c, variant=0), "v1": lambda: gemm_nt(a, b, out=c, variant=1),
               "lib": lambda: torch.matmul(a, b.t(), out=c),
               "fp8_v0": lambda: mx_gemm(qa, sa, qb, sb, out=c, variant=0),
               "fp8_v1": lambda: mx_gemm(qa, sa, qb, sb, out=c, variant=1),
               "mxquant_a": lambda: mx_quantize(a)}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        ts = {k: [] for k in fns}
        for _ in range(rounds):
            for k, f in fns.items():
                ts[k].append(timeit(f, 10))
        fl = 2.0 * M * N * K
        ref = a[:256].float() @ b.float().t()
        errs = {v: (gemm_nt(a[:256], b, variant=v).float() - ref).abs().max().item() for v in (0, 1)}
        rec = {"shape": name, "M": M, "N": N, "K": K, "max_abs_err_256rows": errs}
        full = a[:256].float() @ b.float().t()
        rec["fp8_rel_err_256rows"] = ((mx_gemm(qa[:256], sa[:, :256].contiguous(), qb, sb).float() - full).norm()
                                      / full.norm()).item()
        for k in fns:
            rec[k + "_ms"] = min(ts[k])
            rec[k + "_tflops"] = round(fl / min(ts[k]) / 1e9, 1)
        print(json.dumps(rec), flush=True)
        del a, b, c, qa, qb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
