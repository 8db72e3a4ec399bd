"""qkv projection at the bench shape (T=28672, K=4096, N=6144): one hipBLASLt GEMM vs q (4096) + kv (2048) GEMMs written
into column slices of one output, vs the hand-written MFMA GEMM."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.gemm import gemm_nt  # noqa: E402


def t(fn, it=20):
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
    T, K, N = 28672, 4096, 6144
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    out = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    fl = 2 * T * N * K
    r = {}
    r["fused_ms"] = t(lambda: F.linear(x, w))
    r["split_cat_ms"] = t(lambda: torch.cat([F.linear(x, w[:4096]), F.linear(x, w[4096:])], 1))
    r["split_two_outputs_ms"] = t(lambda: (F.linear(x, w[:4096]), F.linear(x, w[4096:])))
    r["hand_mfma_ms"] = t(lambda: gemm_nt(x, w, out=out))
    r["hand_mfma_v0_ms"] = t(lambda: gemm_nt(x, w, out=out, variant=0))
    print(json.dumps({k: round(v, 4) for k, v in r.items()} | {k.replace("_ms", "_PFs"): round(fl / v / 1e12, 3)
                                                                for k, v in r.items()}))


def slices():
    """The framework's split forward (two GEMMs into column slices of one output) vs fused, at the bench shape."""
    from hcache_deepspeed_amd.runtime.zero.linear import _split_fwd
    T, K, N = 28672, 4096, 6144
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    ref = F.linear(x, w)
    got = _split_fwd(x, w, 4096)
    r32 = x[:4096].float() @ w.float().t()  # both must be bf16 roundings of the same product (reduction order aside)
    e_ref = (ref[:4096].float() - r32).abs().max().item()
    e_got = (got[:4096].float() - r32).abs().max().item()
    print(json.dumps({"err_fused": e_ref, "err_split": e_got}), flush=True)
    assert e_got <= 1.5 * e_ref + 1e-3
    fl = 2 * T * N * K
    r = {"fused_ms": t(lambda: F.linear(x, w)), "split_slices_ms": t(lambda: _split_fwd(x, w, 4096))}
    print(json.dumps({k: round(v, 4) for k, v in r.items()} | {k.replace("_ms", "_PFs"): round(fl / v / 1e12, 3)
                                                                for k, v in r.items()}))


if __name__ == "__main__":
    slices() if "--slices" in sys.argv else main()
