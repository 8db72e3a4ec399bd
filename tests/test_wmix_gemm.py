"""Mixed-input MFMA GEMM (csrc/kernels/wmix_gemm.hip): INT8 / INT4 / FP6 weight-only x bf16 activations against
an fp32 reference of the same op (dequantized weight, fp32 matmul). Reference parity: the CUTLASS mixed GEMM
(K37) and the FP6-LLM linear (K29), whose tests compare against a dequantized fp16 matmul."""
import pytest
import torch

from hcache_deepspeed_amd.ops import quantizer as Q

pytestmark = pytest.mark.gpu


def _ref(x, wq):
    return (x.float() @ wq.float().t())


@pytest.mark.parametrize("fmt", ["int8", "int4", "fp6_e3m2", "fp6_e2m3"])
@pytest.mark.parametrize("M,N,K,G", [(9, 384, 512, 128), (33, 1000, 1024, 32), (64, 4096, 4096, 128),
                                     (100, 520, 768, 64), (200, 256, 2048, 128)])
def test_wmix_matches_dequant_reference(fmt, M, N, K, G):
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    bias = torch.randn(N, device=dev, dtype=torch.bfloat16)
    if fmt.startswith("int"):
        bits = int(fmt[3:])
        q, s, _ = Q.quantize(w.reshape(-1), G, bits, True)
        wd = Q.dequantize(q, s, None, G, bits, True, torch.float32).view(N, K)
        y = Q.wmix_gemm(x, q, s, N, K, G, fmt, bias=bias)
        y2 = Q.int_linear(x, q, s, N, K, G, bits=bits, bias=bias)  # dispatcher takes the same kernel
    else:
        mb = 2 if fmt.endswith("e3m2") else 3
        q, s = Q.quantize_minifloat(w.reshape(-1), G, 6, mb)
        wd = Q.dequantize_minifloat(q, s, G, 6, mb, torch.float32).view(N, K)
        y = Q.wmix_gemm(x, q, s, N, K, G, "fp6", 5 - mb, bias=bias)
        y2 = Q.fp6_linear(x, q, s, N, K, G, mb) + bias
    ref = _ref(x, wd) + bias.float()
    err = (y.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    # bf16 rounding of the dequantized weight (8 bits) + bf16 output: ~1e-2 relative of the largest output
    assert err <= 1e-2 * scale + 1e-2, (fmt, M, N, K, G, err, scale)
    assert (y2.float() - ref).abs().max().item() <= 1.5e-2 * scale + 2e-2


def test_wmix_split_k_deterministic():
    torch.manual_seed(1)
    x = torch.randn(48, 14336, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(512, 14336, device="cuda", dtype=torch.bfloat16) * 0.02
    q, s, _ = Q.quantize(w.reshape(-1), 128, 8, True)
    from hcache_deepspeed_amd.ops import native
    assert native.kernels().hds_wmix_splits(48, 512, 14336) > 1
    a = Q.wmix_gemm(x, q, s, 512, 14336, 128, "int8")
    b = Q.wmix_gemm(x, q, s, 512, 14336, 128, "int8")
    assert torch.equal(a, b)
    ref = x.float() @ Q.dequantize(q, s, None, 128, 8, True, torch.float32).view(512, 14336).t()
    assert (a.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
