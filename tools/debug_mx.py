"""Probe the MX-FP8 GEMM operand mapping with exact data (one-hot A rows, integer B, unit / patterned scales)."""
import sys

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops.fp8_gemm import mx_dequantize, mx_gemm  # noqa: E402


def e4m3(t):
    return t.float().to(torch.float8_e4m3fn).view(torch.uint8)


M = N = K = 256
dev = "cuda"
# test 1: unit scales, A one-hot (A[m, m] = 1), B[n, k] = (k % 13) - 6  -> C[m, n] = B[n, m]
qa = e4m3(torch.eye(M, K)).to(dev)
b = torch.tensor([[((k * 7 + n) % 13) - 6 for k in range(K)] for n in range(N)], dtype=torch.float32)
qb = e4m3(b).to(dev)
s1 = torch.full((K // 128, M, 4), 127, dtype=torch.uint8, device=dev)
c = mx_gemm(qa, s1, qb, s1.clone()).float().cpu()
ref = b.t()  # C[m, n] = b[n, m]
bad = (c != ref).any(1)
print("test1 unit-scale one-hot: rows wrong", int(bad.sum()), "of", M)
# for wrong rows: which k of B does row m actually pick?
bt = b.t()  # [k, n]
for m in [i for i in range(M) if bad[i]][:12]:
    hits = [k for k in range(K) if torch.equal(c[m], bt[k])]
    print(f"  row {m}: matches B column k={hits}  (sum={c[m].abs().sum().item():.1f})")
# test 2: all-ones data, scale of block (r, g) = 127 + (g % 4) for A, 127 for B -> C = sum_g 32 * 2^(g%4)
ones = e4m3(torch.ones(M, K)).to(dev)
sa = torch.full((K // 128, M, 4), 127, dtype=torch.uint8)
for t in range(K // 128):
    for g in range(4):
        sa[t, :, g] = 127 + g + 4 * t
sa = sa.to(dev)
c2 = mx_gemm(ones, sa, ones, s1.clone()).float().cpu()
ref2 = (mx_dequantize(ones.cpu(), sa.cpu()) @ mx_dequantize(ones.cpu(), s1.cpu()).t())
print("test2 A block scales: got", c2[0, :4].tolist(), "ref", ref2[0, :4].tolist())
sb = sa.clone()
c3 = mx_gemm(ones, s1.clone(), ones, sb).float().cpu()
print("test3 B block scales: got", c3[0, :4].tolist(), "ref", ref2[0, :4].tolist())
# test 4: per-row A scale (row m -> 127 + m % 5)
sr = torch.full((K // 128, M, 4), 127, dtype=torch.uint8)
for m in range(M):
    sr[:, m, :] = 127 + (m % 5)
c4 = mx_gemm(ones, sr.to(dev), ones, s1.clone()).float().cpu()
ref4 = mx_dequantize(ones.cpu(), sr) @ mx_dequantize(ones.cpu(), s1.cpu()).t()
print("test4 row scales: got", c4[:6, 0].tolist(), "ref", ref4[:6, 0].tolist())
# test 5: which lane-group scale applies to memory position k0? row m one-hot at k0 = m % 128, A block scales
# 127 + g (g = 0..3 per K-tile), B ones with unit scales -> C[m, 0] = 2**g_applied
a5 = torch.zeros(M, K)
for m in range(M):
    a5[m, m % 128] = 1
q5 = e4m3(a5).to(dev)
c5 = mx_gemm(q5, sa, ones, s1.clone()).float().cpu()
applied = torch.log2(c5[:128, 0]).round().int().tolist()
print("test5 k0 -> applied block:", applied)
