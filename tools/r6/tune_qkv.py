"""TunableOp over the one GEMM shape hipBLASLt's heuristic leaves at 64 % MFMA busy (profiles/r6/gemm_pmc_hipblaslt_r6.txt):
the qkv projection forward F.linear([28672, 4096], [6144, 4096]) of the headline step. Times the heuristic pick, tunes
(hipBLASLt + rocBLAS candidates), times the tuned pick; the table lands in $PYTORCH_TUNABLEOP_FILENAME."""
import json
import os
import sys

import torch
import torch.nn.functional as F

shapes = [(28672, 4096, 6144)] + ([(28672, 4096, 4096)] if "--o" in sys.argv else [])


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


tun = torch.cuda.tunable
for M, K, N in shapes:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    tun.enable(False)
    base = timeit(lambda: F.linear(x, w))
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(60)
    F.linear(x, w)  # tunes this signature
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    tuned = timeit(lambda: F.linear(x, w))
    fl = 2 * M * N * K
    print(json.dumps({"M": M, "K": K, "N": N, "heuristic_ms": round(base, 4), "tuned_ms": round(tuned, 4),
                      "heuristic_tflops": round(fl / base / 1e9, 1), "tuned_tflops": round(fl / tuned / 1e9, 1),
                      "results": [list(map(str, r)) for r in (tun.get_results() or ())]}),  # tuple of rows
          flush=True)
tun.write_file()
print("wrote", tun.get_filename())
