"""Channels-last (NHWC) bias-add fusions for diffusion UNet / VAE blocks.

Reference parity: ops/spatial (``nhwc_bias_add``; csrc/spatial/csrc/opt_bias_add.cu). One HIP
pass (csrc/kernels/token_ops.hip ``nhwc_bias_add_kernel``) computes ``a + bias [+ other [+ other_bias]]`` with the
channel dimension innermost; CPU tensors use the torch expression.
"""
import torch

from . import native


def nhwc_bias_add(activation, bias, other=None, other_bias=None):
    """activation / other: [N, H, W, C] (or any [..., C] contiguous); bias / other_bias: [C]."""
    C = activation.shape[-1]
    if not (native.use_native(activation) and C % 8 == 0 and activation.is_contiguous()
            and activation.dtype in (torch.float32, torch.bfloat16, torch.float16)):
        out = activation + bias
        if other is not None:
            out = out + other
            if other_bias is not None:
                out = out + other_bias
        return out
    mode = 0 if other is None else (1 if other_bias is None else 2)
    bias = bias.to(activation.dtype).contiguous()
    if other is not None:
        other = other.to(activation.dtype).contiguous()
        assert other.shape == activation.shape
    if other_bias is not None:
        other_bias = other_bias.to(activation.dtype).contiguous()
    assert bias.numel() == C
    out = torch.empty_like(activation)
    native.check(native.kernels().hds_nhwc_bias_add(native.dt(activation), activation.data_ptr(), bias.data_ptr(),
                                                     native.ptr(other), native.ptr(other_bias), out.data_ptr(),
                                                     activation.numel() // C, C, mode, native.stream()),
                 "nhwc_bias_add")
    return out
