"""Micro-benchmark: SwiGLU forward/backward kernels at the Llama-3-8B bench shape (mb7 x 4096 tokens,
I = 14336), reported as time and effective HBM bandwidth. Earlier kernel (profiles/rocprof_kernel_stats_r1_mb7.csv):
glu_fwd 473 us, glu_bwd 839 us."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hcache_deepspeed_amd.ops import native  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    lib = native.kernels()
    T, I = 7 * 4096, 14336
    gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(T, I, device="cuda", dtype=torch.bfloat16)
    dgu = torch.empty_like(gu)
    st = native.stream()
    dt = native.dt(gu)
    fwd = timeit(lambda: lib.hds_glu_fwd(dt, 0, gu.data_ptr(), y.data_ptr(), T, I, st))
    bwd = timeit(lambda: lib.hds_glu_bwd(dt, 0, dy.data_ptr(), gu.data_ptr(), dgu.data_ptr(), T, I, st))
    yt = torch.empty(I, T, device="cuda", dtype=torch.bfloat16)
    dgut = torch.empty(2 * I, T, device="cuda", dtype=torch.bfloat16)
    fwd_t = timeit(lambda: lib.hds_glu_fwd_t(0, gu.data_ptr(), y.data_ptr(), yt.data_ptr(), T, I, st))
    bwd_t = timeit(lambda: lib.hds_glu_bwd_t(0, dy.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dgut.data_ptr(), T, I,
                                             st))
    # numerics vs fp32 torch
    g, u = gu.float().chunk(2, -1)
    ref = torch.nn.functional.silu(g) * u
    err_f = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    s = torch.sigmoid(g)
    ref_dg = dy.float() * u * s * (1 + g * (1 - s))
    err_b = ((dgu[:, :I].float() - ref_dg).abs().max() / ref_dg.abs().max()).item()
    el = T * I * 2
    print(json.dumps({"T": T, "I": I, "glu_fwd_us": round(fwd, 1), "glu_fwd_TBps": round(3 * el / fwd / 1e6, 2),
                      "glu_bwd_us": round(bwd, 1), "glu_bwd_TBps": round(5 * el / bwd / 1e6, 2),
                      "glu_fwd_t_us": round(fwd_t, 1), "glu_fwd_t_TBps": round(4 * el / fwd_t / 1e6, 2),
                      "glu_bwd_t_us": round(bwd_t, 1), "glu_bwd_t_TBps": round(7 * el / bwd_t / 1e6, 2),
                      "variant": os.environ.get("HDS_GLU_VAR", "2"),
                      "rel_err_fwd": err_f, "rel_err_bwd_dgate": err_b}))


if __name__ == "__main__":
    main()
