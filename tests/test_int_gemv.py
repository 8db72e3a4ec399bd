"""Weight-only INT8/INT4 linear (csrc/kernels/quant.hip ``int_gemv_kernel`` for decode, dequantize + GEMM for prefill)
against an fp32 torch reference of the dequantized weight (reference tests/unit/inference/quantization)."""
import pytest
import torch

from hcache_deepspeed_amd.ops import quantizer as Q


def _case(device, M, bits, N=384, K=512, G=128):
    torch.manual_seed(M * 10 + bits)
    w = torch.randn(N, K, device=device, dtype=torch.bfloat16) * 0.05
    q, s, _ = Q.quantize(w.reshape(-1).contiguous(), G, bits, True)
    x = torch.randn(M, K, device=device, dtype=torch.bfloat16)
    bias = torch.randn(N, device=device, dtype=torch.bfloat16)
    y = Q.int_linear(x, q, s, N, K, G, bits, bias)
    wd = Q.dequantize(q, s, None, G, bits, True, torch.float32).view(N, K)
    ref = x.float() @ wd.t() + bias.float()
    return y, ref, wd, w


@pytest.mark.parametrize("bits", [8, 4])
def test_int_linear_cpu(bits):
    y, ref, wd, w = _case("cpu", 3, bits)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    assert (wd - w.float()).abs().max() < (0.02 if bits == 8 else 0.2)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [8, 4])
@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("N", [384, 16384])
def test_int_linear_hip(cuda, M, bits, N, monkeypatch):
    monkeypatch.setattr(Q, "_INT_GEMV_MAX_M", 8)  # exercise every fused template, not just the default M <= 2
    y, ref, _, _ = _case(cuda, M, bits, N=N)
    assert y.shape == ref.shape and y.dtype == torch.bfloat16
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)
