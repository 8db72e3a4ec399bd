"""FP6 / FP12 minifloat quantization (fpq.hip) and the FP6 weight-only GEMV.

Reference test analogue: tests/unit/ops/fp_quantizer/test_fp_quant.py (quantize -> dequantize vs a reference
within format error, q_bits in {8, 6, 12}, stochastic rounding) and tests/unit/inference/v2/kernels/core_ops/
(FP6 linear). Numerics reference: the torch encoder in ops/quantizer.py (exact code-level comparison on GPU).
"""
import pytest
import torch

from hcache_deepspeed_amd.ops import quantizer as Q


@pytest.mark.parametrize("q_bits,m", [(6, 2), (6, 3), (12, 7), (8, 3)])
def test_codes_roundtrip_exhaustive(q_bits, m):
    codes = torch.arange(2**q_bits)
    vals = Q._ref_decode(codes, q_bits, m)
    back = Q._ref_encode(vals, q_bits, m)
    # +0 / -0 both decode to 0
    nz = vals != 0
    assert torch.equal(back[nz], codes[nz].to(back.dtype))
    _, _, maxval = Q._mini_fmt(q_bits, m)
    assert float(vals.abs().max()) == maxval


@pytest.mark.parametrize("q_bits,m", [(6, 2), (12, 7)])
def test_quant_dequant_error_and_packing(q_bits, m):
    torch.manual_seed(0)
    x = torch.randn(4 * 512)
    q, s = Q.quantize_minifloat(x, 512, q_bits, m)
    assert q.numel() == x.numel() * q_bits // 8 and q.dtype == torch.uint8
    y = Q.dequantize_minifloat(q, s, 512, q_bits, m, torch.float32)
    rel = ((y - x).norm() / x.norm()).item()
    assert rel < (0.12 if q_bits == 6 else 0.005), rel
    # nearest rounding: every value is the nearest representable point
    grid = Q._ref_decode(torch.arange(2**q_bits), q_bits, m).unique()
    xs = (x.reshape(4, -1) / s[:, None]).reshape(-1)
    ys = (y.reshape(4, -1) / s[:, None]).reshape(-1)
    best = grid[(xs[:, None] - grid[None]).abs().argmin(1)]
    assert torch.allclose(ys, best, atol=1e-6)


def test_fp_quantize_api_fp6_fp12_and_stochastic():
    torch.manual_seed(1)
    fq = Q.FP_Quantize(group_size=128)
    x = torch.randn(8, 256)
    q = fq.quantize(x, q_bits=6, q_mantisa_bits=2)
    y = fq.dequantize(q, q_bits=6, q_mantisa_bits=2)
    assert y.shape == x.shape and ((y.float() - x).norm() / x.norm()) < 0.12
    rows = fq.selective_dequantize(q, torch.tensor([1, 5]), q_bits=6, q_mantisa_bits=2)
    assert torch.allclose(rows.float(), y[[1, 5]].float())
    q12 = fq.quantize(x, q_bits=12, q_mantisa_bits=7)
    assert ((fq.dequantize(q12, q_bits=12, q_mantisa_bits=7).float() - x).norm() / x.norm()) < 0.005
    # stochastic rounding is unbiased: the mean of many draws approaches x
    xv = torch.full((512, ), 0.3)
    xv[0] = 1.0  # fixes the scale
    acc = torch.zeros(512)
    for seed in range(200):
        qq, ss = Q.quantize_minifloat(xv, 512, 6, 2, stochastic=True, seed=seed)
        acc += Q.dequantize_minifloat(qq, ss, 512, 6, 2, torch.float32)
    assert abs(acc[1:].mean().item() / 200 - 0.3) < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("q_bits,m,dtype", [(6, 2, torch.bfloat16), (6, 3, torch.float32), (12, 7, torch.bfloat16),
                                            (8, 3, torch.float16)])
def test_minifloat_kernel_matches_reference(q_bits, m, dtype):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(2)
    x = (torch.randn(64 * 256) * 3).to(dtype)
    qg, sg = Q.quantize_minifloat(x.cuda(), 256, q_bits, m)
    qc, sc = Q.quantize_minifloat(x, 256, q_bits, m)
    torch.cuda.synchronize()
    assert torch.allclose(sg.cpu(), sc, rtol=1e-6)
    assert torch.equal(qg.cpu(), qc), "packed codes must match the reference encoder bit for bit"
    yg = Q.dequantize_minifloat(qg, sg, 256, q_bits, m, dtype)
    yc = Q.dequantize_minifloat(qc, sc, 256, q_bits, m, dtype)
    assert torch.equal(yg.cpu(), yc)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 8, 32])
def test_fp6_linear_gpu(M):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(3)
    N, K, G = 1024, 2048, 128
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    qw, sw = Q.quantize_minifloat(w.reshape(-1), G, 6, 2)
    wd = Q.dequantize_minifloat(qw, sw, G, 6, 2, torch.float32).view(N, K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    y = Q.fp6_linear(x, qw, sw, N, K, G)
    ref = x.float() @ wd.t()
    torch.cuda.synchronize()
    assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-2


def test_quantized_linear_fp6_cpu():
    from hcache_deepspeed_amd.linear.config import QuantizationConfig
    from hcache_deepspeed_amd.linear.quantization import QuantizedLinear
    torch.manual_seed(4)
    ql = QuantizedLinear(256, 64, quantization_config=QuantizationConfig(q_bits=6, mantissa_bits=2, group_size=128),
                         dtype=torch.float32)
    w = ql.weight.dequantized()
    assert w.shape == (64, 256) and ql.weight.q_data.numel() == 64 * 256 * 6 // 8
    x = torch.randn(3, 256)
    assert torch.allclose(ql(x), x @ w.t(), atol=1e-5)
