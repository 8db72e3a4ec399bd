"""Gate/up backward layouts at the bench shape (T=28672, I=14336, H=4096): would a GLU backward that writes dH^T
(instead of dH) pay? Times the current path (dgrad on dH + wgrad via transposes) against GEMMs fed dH^T directly."""
import json

import torch

from hcache_deepspeed_amd.ops.gemm import dgrad, transpose2d, wgrad


def timeit(fn, it=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    T, N, K = 28672, 28672, 4096
    dh = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.01
    dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    dx = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
    dht = transpose2d(dh)
    wt = transpose2d(w)
    xt = transpose2d(x)
    r = {}
    r["transpose_dh_ms"] = timeit(lambda: transpose2d(dh))
    r["transpose_x_ms"] = timeit(lambda: transpose2d(x))
    r["cur_dgrad_ms"] = timeit(lambda: dgrad(dh, w, out=dx))
    r["cur_wgrad_ms"] = timeit(lambda: wgrad(dh, x, dw))
    r["dgrad_from_dhT_NN_ms"] = timeit(lambda: torch.mm(dht.t(), w, out=dx))
    r["dgrad_from_dhT_wT_ms"] = timeit(lambda: torch.mm(dht.t(), wt.t(), out=dx))
    r["wgrad_from_dhT_xT_ms"] = timeit(lambda: torch.mm(dht, xt.t(), out=dw))
    r["wgrad_from_dhT_x_ms"] = timeit(lambda: torch.mm(dht, x, out=dw))
    print(json.dumps({k: round(v, 3) for k, v in r.items()}))


if __name__ == "__main__":
    main()
