"""Memory-efficient linear for ZeRO-3 (reference runtime/zero/linear.py ``LinearFunctionForZeroStage3`` :50).

A plain ``F.linear`` saves the weight TENSOR for backward, which pins the gathered full buffer of the whole
unit until the backward pass -- a partitioned model would keep every layer's gathered weights alive. This
Function saves only the input and keeps a reference to the Parameter OBJECT; by the time its backward runs
the unit has been re-gathered (pre-backward hook) and ``weight.data`` points at the new full buffer, so the
forward copy can be freed right after the layer's forward.
"""
import types

import torch
import torch.nn as nn
import torch.nn.functional as F


class LinearFunctionForZeroStage3(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, weight, bias=None):
        ctx.save_for_backward(x)
        ctx.weight = weight
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        (x, ) = ctx.saved_tensors
        w = ctx.weight
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = dy.matmul(w.to(dy.dtype))
        if ctx.needs_input_grad[1]:
            dw = dy.reshape(-1, dy.shape[-1]).t().matmul(x.reshape(-1, x.shape[-1]).to(dy.dtype))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).sum(0)
        return dx, dw, db


def zero3_linear(x, weight, bias=None):
    return LinearFunctionForZeroStage3.apply(x, weight, bias)


def _mel_forward(self, x):
    return zero3_linear(x, self.weight, self.bias)


def wrap_memory_efficient_linears(module):
    """Route every nn.Linear under ``module`` through the memory-efficient Function (instance-level)."""
    n = 0
    for m in module.modules():
        if isinstance(m, nn.Linear) and not getattr(m, "_hds_mel", False):
            m.forward = types.MethodType(_mel_forward, m)
            m._hds_mel = True
            n += 1
    return n
