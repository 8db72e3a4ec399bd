"""OptimizedLinear / LoRA / FP8 QuantizedLinear (reference tests/unit/linear/test_linear.py, test_quant_param.py)."""
import pytest
import torch

from tests.dist_utils import run_distributed


def test_lora_linear_forward_and_grads():
    from hcache_deepspeed_amd.linear import LoRAConfig, OptimizedLinear
    torch.manual_seed(0)
    lin = OptimizedLinear(32, 48, lora_config=LoRAConfig(lora_r=4, lora_alpha=8), dtype=torch.float32)
    x = torch.randn(5, 32)
    y = lin(x)
    assert torch.allclose(y, x @ lin.full_weight().t(), atol=1e-5)  # B = 0 at init
    y.sum().backward()
    assert lin.weight.grad is None and not lin.weight.requires_grad
    assert lin.lora_weight_2.weight.grad is not None
    with torch.no_grad():
        lin.lora_weight_2.weight.normal_()
    y1 = lin(x)
    lin.fuse_lora_weight()
    assert torch.allclose(lin(x), y1, atol=1e-4)
    lin.unfuse_lora_weight()
    assert torch.allclose(lin(x), y1, atol=1e-4)


def test_plain_and_quantized_dispatch():
    import torch.nn as nn
    from hcache_deepspeed_amd.linear import OptimizedLinear, QuantizationConfig, QuantizedLinear
    assert type(OptimizedLinear(8, 8, dtype=torch.float32)) is nn.Linear
    q = OptimizedLinear(64, 64, quantization_config=QuantizationConfig(group_size=64), dtype=torch.float32)
    assert isinstance(q, QuantizedLinear)
    x = torch.randn(3, 64)
    w = q.weight.dequantized()
    assert w.shape == (64, 64) and torch.allclose(q(x), x @ w.t(), atol=1e-5)


def _sharded(rank, world):
    from hcache_deepspeed_amd.linear import LoRAConfig, OptimizedLinear
    torch.manual_seed(0)  # same init on both ranks -> shards of one weight
    lin = OptimizedLinear(30, 20, lora_config=LoRAConfig(lora_r=2, base_weight_sharding=world), dtype=torch.float32)
    assert lin.weight.numel() == (30 * 20 + world - 1) // world
    full = lin.full_weight()
    torch.manual_seed(0)
    ref = OptimizedLinear(30, 20, lora_config=LoRAConfig(lora_r=2), dtype=torch.float32)
    assert torch.equal(full, ref.full_weight())


def test_base_weight_sharding_world2():
    run_distributed(_sharded, 2)


def test_quantized_linear_mx_fp8_cpu_reference():
    """8-bit e4m3 QuantizedLinear with mx_fp8 keeps an MX-FP8 copy derived from the quantized weight; off-GPU it
    runs the dequantized MX weight. The default is the reference's weight-only path."""
    from hcache_deepspeed_amd.linear import QuantizationConfig
    from hcache_deepspeed_amd.linear.quantization import QuantizedLinear
    from hcache_deepspeed_amd.ops.fp8_gemm import mx_dequantize
    torch.manual_seed(0)
    ql = QuantizedLinear(512, 256, quantization_config=QuantizationConfig(q_bits=8, group_size=128, mx_fp8=True),
                         dtype=torch.float32)
    assert ql.weight.mx_ok() and ql.weight.mx_shape == (256, 512)
    x = torch.randn(4, 512)
    w = mx_dequantize(*ql.weight.mx_w)
    torch.testing.assert_close(ql(x), x @ w.t())
    off = QuantizedLinear(512, 256, quantization_config=QuantizationConfig(q_bits=8, group_size=128),
                          dtype=torch.float32)
    assert not off.weight.mx_ok()  # default: weight-only
    torch.testing.assert_close(off(x), x @ off.weight.dequantized().float().t())
    # the MX copy tracks re-quantization (no stale snapshot)
    ql.weight._ensure_quantized(torch.randn(256, 512))
    torch.testing.assert_close(mx_dequantize(*ql.weight.mx_w).float(),
                               mx_dequantize(*__import__("hcache_deepspeed_amd.ops.fp8_gemm", fromlist=["x"]).mx_quantize(
                                   ql.weight.dequantized().reshape(256, 512).to(torch.bfloat16))).float())


def test_quantized_fp6_lora_base_passes_input_gradient():
    """a frozen FP6 base under LoRA training must pass dX to earlier layers at every token count."""
    from hcache_deepspeed_amd.linear import QuantizationConfig
    from hcache_deepspeed_amd.linear.quantization import QuantizedLinear
    torch.manual_seed(0)
    ql = QuantizedLinear(256, 128, quantization_config=QuantizationConfig(q_bits=6, mantissa_bits=2, group_size=64),
                         dtype=torch.float32)
    for rows in (1, 9, 64, 300):
        x = torch.randn(rows, 256, requires_grad=True)
        ql(x).sum().backward()
        assert x.grad is not None and x.grad.abs().sum() > 0, rows
