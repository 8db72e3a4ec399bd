"""Gated activations (SwiGLU/GeGLU/ReGLU) and bias+activation, HIP fwd/bwd.

Reference parity: inference/v2/kernels/core_ops/gated_activations (CUDAGatedActivation) and
bias_activations (CUDABiasActivation); training GeLU of csrc/transformer/gelu_kernels.cu.
"""
import torch
import torch.nn.functional as F

from . import native
from ..offload import act_plan as _ap

SILU, GELU_TANH, RELU, GELU, IDENTITY = 0, 1, 2, 3, 4
_NAMES = {"silu": SILU, "swish": SILU, "gelu_tanh": GELU_TANH, "gelu_new": GELU_TANH, "gelu_pytorch_tanh": GELU_TANH,
          "relu": RELU, "gelu": GELU, "identity": IDENTITY}


def act_code(name):
    return name if isinstance(name, int) else _NAMES[name]


def _ref_act(x, a):
    if a == SILU:
        return F.silu(x)
    if a == GELU_TANH:
        return F.gelu(x, approximate="tanh")
    if a == RELU:
        return F.relu(x)
    if a == GELU:
        return F.gelu(x)
    return x


def _t_ok(gu):
    """The transposed-output kernels' contract: bf16 on the GPU, rows and I multiples of 8, 16-B aligned."""
    I = gu.shape[-1] // 2
    rows = gu.numel() // max(1, 2 * I)
    return (native.use_native(gu) and gu.dtype == torch.bfloat16 and gu.is_contiguous() and rows % 8 == 0
            and I % 8 == 0 and rows > 0 and gu.data_ptr() % 16 == 0)


def _glu_out(gu, act):
    I = gu.shape[-1] // 2
    if native.use_native(gu):
        gu2 = gu.reshape(-1, 2 * I).contiguous()
        y = torch.empty(gu2.shape[0], I, device=gu.device, dtype=gu.dtype)
        native.check(native.kernels().hds_glu_fwd(native.dt(gu), act, gu2.data_ptr(), y.data_ptr(), gu2.shape[0], I,
                                                  native.stream()), "glu_fwd")
        return y.view(*gu.shape[:-1], I)
    g, u = gu.float().split(I, dim=-1)
    return (_ref_act(g, act) * u).to(gu.dtype)


def _glu_t_recompute(gu, act):
    """The transposed SwiGLU output [I, rows] the down projection saved (per-tensor activation plan recipe)."""
    I = gu.shape[-1] // 2
    rows = gu.numel() // (2 * I)
    y = torch.empty(rows, I, device=gu.device, dtype=gu.dtype)
    yt = torch.empty(I, rows, device=gu.device, dtype=gu.dtype)
    native.check(native.kernels().hds_glu_fwd_t(act, gu.data_ptr(), y.data_ptr(), yt.data_ptr(), rows, I,
                                                native.stream()), "glu_fwd_t")
    return yt


class _GLUFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, gu, act, transposed=False):
        I = gu.shape[-1] // 2
        ctx.act = act
        ctx.save_for_backward(gu)
        ctx.transposed = bool(transposed) and _t_ok(gu)
        if ctx.transposed:
            rows = gu.numel() // (2 * I)
            y = torch.empty(rows, I, device=gu.device, dtype=gu.dtype)
            yt = torch.empty(I, rows, device=gu.device, dtype=gu.dtype)
            native.check(native.kernels().hds_glu_fwd_t(act, gu.data_ptr(), y.data_ptr(), yt.data_ptr(), rows, I,
                                                        native.stream()), "glu_fwd_t")
            out = y.view(*gu.shape[:-1], I)
            out._hds_t = yt  # the consumer may save this [I, rows] copy instead of out (runtime/zero/linear.py)
            if _ap.tracking():
                _ap.tag(yt, "glu_t", fn=_glu_t_recompute, srcs=(gu, act))
            return out
        y = _glu_out(gu, act)
        if _ap.tracking():
            _ap.tag(y, "glu_out", fn=_glu_out, srcs=(gu, act))
        return y

    @staticmethod
    def backward(ctx, dy):
        (gu, ) = ctx.saved_tensors
        I = gu.shape[-1] // 2
        if ctx.transposed and dy.dtype == gu.dtype:
            from .gemm import wants_transposed_dy
            if wants_transposed_dy(2 * I):
                rows = gu.numel() // (2 * I)
                d = dy.reshape(rows, I).contiguous()
                dgu = torch.empty(rows, 2 * I, device=gu.device, dtype=gu.dtype)
                dgut = torch.empty(2 * I, rows, device=gu.device, dtype=gu.dtype)
                native.check(native.kernels().hds_glu_bwd_t(ctx.act, d.data_ptr(), gu.data_ptr(), dgu.data_ptr(),
                                                            dgut.data_ptr(), rows, I, native.stream()), "glu_bwd_t")
                r = dgu.view(gu.shape)
                r._hds_t = dgut  # the gate|up projection's weight gradient reads this [2I, rows] copy (NT form)
                return r, None, None
        if native.use_native(gu):
            gu2 = gu.reshape(-1, 2 * I).contiguous()
            dgu = torch.empty_like(gu2)
            native.check(native.kernels().hds_glu_bwd(native.dt(gu), ctx.act, dy.reshape(-1, I).contiguous().data_ptr(),
                                                      gu2.data_ptr(), dgu.data_ptr(), gu2.shape[0], I,
                                                      native.stream()), "glu_bwd")
            return dgu.view(gu.shape), None, None
        with torch.enable_grad():
            g = gu.detach().float().requires_grad_(True)
            a, u = g.split(I, dim=-1)
            y = _ref_act(a, ctx.act) * u
            (dg, ) = torch.autograd.grad(y, g, dy.float())
        return dg.to(gu.dtype), None, None


def glu(gu, act="silu", transposed=False):
    """act(gu[..., :I]) * gu[..., I:] for the fused gate|up projection output.

    ``transposed=True`` (bf16 on the GPU, rows % 8 == 0): the kernel also writes the output's transpose [I, rows]
    and attaches it as ``out._hds_t``; a ZeRO linear consuming ``out`` saves that copy instead of ``out`` for its
    weight gradient (hipBLASLt's NT form needs the token dimension contiguous). The backward likewise hands the
    gate|up projection the transpose of d(gate|up). Both replace a separate HBM transpose pass in the backward."""
    return _GLUFn.apply(gu, act_code(act), bool(transposed))


def swiglu(gu):
    return _GLUFn.apply(gu, SILU, False)


class _BiasActFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, bias, act):
        ctx.act = act
        ctx.save_for_backward(x, bias)
        C = x.shape[-1]
        if native.use_native(x):
            x2 = x.reshape(-1, C).contiguous()
            y = torch.empty_like(x2)
            native.check(native.kernels().hds_bias_act_fwd(native.dt(x), act, x2.data_ptr(), native.ptr(bias),
                                                           y.data_ptr(), x2.shape[0], C, native.stream()), "bias_act")
            return y.view(x.shape)
        xf = x.float() + (bias.float() if bias is not None else 0.0)
        return _ref_act(xf, act).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        C = x.shape[-1]
        if native.use_native(x):
            x2 = x.reshape(-1, C).contiguous()
            dx = torch.empty_like(x2)
            native.check(native.kernels().hds_bias_act_bwd(native.dt(x), ctx.act, dy.reshape(-1, C).contiguous().data_ptr(),
                                                           x2.data_ptr(), native.ptr(bias), dx.data_ptr(), x2.shape[0],
                                                           C, native.stream()), "bias_act_bwd")
            dx = dx.view(x.shape)
        else:
            with torch.enable_grad():
                xf = (x.detach().float() + (bias.float() if bias is not None else 0.0)).requires_grad_(True)
                (dxf, ) = torch.autograd.grad(_ref_act(xf, ctx.act), xf, dy.float())
            dx = dxf.to(x.dtype)
        db = dx.reshape(-1, C).float().sum(0).to(bias.dtype) if bias is not None else None
        return dx, db, None


def bias_act(x, bias=None, act="gelu"):
    return _BiasActFn.apply(x, bias, act_code(act))
