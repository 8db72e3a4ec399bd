"""Host (CPU) optimizers for ZeRO-Offload: DeepSpeedCPUAdam / DeepSpeedCPULion / DeepSpeedCPUAdagrad.

Reference parity: ops/adam/cpu_adam.py:13 (``DeepSpeedCPUAdam``, fp16/bf16 param output, AVX-512/AVX2 +
OpenMP), ops/lion/cpu_lion.py:13, ops/adagrad/cpu_adagrad.py:11. Kernels: csrc/host/cpu_optim.cpp.
"""
import torch

from . import native


def _gd(t):
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    raise TypeError(f"cpu optimizers take fp32/bf16 grads, got {t.dtype}")


def cpu_adam_flat(p, g, m, v, step, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=True,
                  bias_correction=True, bf16_out=None, grad_scale=1.0):
    assert p.dtype == torch.float32 and p.is_contiguous() and not p.is_cuda
    b1, b2 = betas
    bc1 = 1 - b1**step if bias_correction else 1.0
    bc2 = 1 - b2**step if bias_correction else 1.0
    native.check(
        native.host_lib().hds_cpu_adam(p.data_ptr(), g.data_ptr(), _gd(g), m.data_ptr(), v.data_ptr(),
                                       bf16_out.data_ptr() if bf16_out is not None else None, p.numel(), float(lr),
                                       float(b1), float(b2), float(eps), float(weight_decay), float(bc1), float(bc2),
                                       int(adamw), float(grad_scale)), "cpu_adam")


def cpu_lion_flat(p, g, m, lr, betas=(0.9, 0.99), weight_decay=0.0, bf16_out=None, grad_scale=1.0):
    b1, b2 = betas
    native.check(
        native.host_lib().hds_cpu_lion(p.data_ptr(), g.data_ptr(), _gd(g), m.data_ptr(),
                                       bf16_out.data_ptr() if bf16_out is not None else None, p.numel(), float(lr),
                                       float(b1), float(b2), float(weight_decay), float(grad_scale)), "cpu_lion")


def cpu_adagrad_flat(p, g, s, lr, eps=1e-10, weight_decay=0.0, bf16_out=None, grad_scale=1.0):
    native.check(
        native.host_lib().hds_cpu_adagrad(p.data_ptr(), g.data_ptr(), _gd(g), s.data_ptr(),
                                          bf16_out.data_ptr() if bf16_out is not None else None, p.numel(),
                                          float(lr), float(eps), float(weight_decay), float(grad_scale)),
        "cpu_adagrad")


def cpu_sumsq(g, found_inf=None):
    import ctypes
    flag = ctypes.c_int(0)
    r = native.host_lib().hds_cpu_sumsq(g.data_ptr(), _gd(g), g.numel(), ctypes.addressof(flag))
    if found_inf is not None:
        found_inf[0] = found_inf[0] or bool(flag.value)
    return r


class DeepSpeedCPUAdam(torch.optim.Optimizer):
    """Adam/AdamW on host fp32 parameters (reference ops/adam/cpu_adam.py:13)."""

    optimizer_id = 0

    def __init__(self, model_params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, adamw_mode=True, fp32_optimizer_states=True):
        if amsgrad:
            raise RuntimeError("DeepSpeedCPUAdam does not support AMSGrad")
        super().__init__(model_params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                            bias_correction=bias_correction, amsgrad=amsgrad))
        self.adam_w_mode = adamw_mode
        self.opt_id = DeepSpeedCPUAdam.optimizer_id
        DeepSpeedCPUAdam.optimizer_id += 1

    @torch.no_grad()
    def step(self, closure=None, fp16_param_groups=None):
        loss = closure() if closure is not None else None
        for gi, group in enumerate(self.param_groups):
            for pi, p in enumerate(group["params"]):
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                st["step"] += 1
                out = None
                if fp16_param_groups is not None:
                    out = fp16_param_groups[gi][pi] if isinstance(fp16_param_groups[gi], (list, tuple)) \
                        else fp16_param_groups[gi]
                cpu_adam_flat(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], st["step"], group["lr"],
                              group["betas"], group["eps"], group["weight_decay"], self.adam_w_mode,
                              group["bias_correction"], bf16_out=out)
        return loss


class DeepSpeedCPULion(torch.optim.Optimizer):

    def __init__(self, model_params, lr=1e-3, betas=(0.9, 0.999), weight_decay=0, fp32_optimizer_states=True):
        super().__init__(model_params, dict(lr=lr, betas=betas, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None, fp16_param_groups=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                cpu_lion_flat(p.data, p.grad.contiguous(), st["exp_avg"], group["lr"], group["betas"],
                              group["weight_decay"])
        return loss


class DeepSpeedCPUAdagrad(torch.optim.Optimizer):

    def __init__(self, model_params, lr=1e-2, eps=1e-10, weight_decay=0, amsgrad=False, fp32_optimizer_states=True):
        super().__init__(model_params, dict(lr=lr, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None, fp16_param_groups=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                cpu_adagrad_flat(p.data, p.grad.contiguous(), st["exp_avg_sq"], group["lr"], group["eps"],
                                 group["weight_decay"])
        return loss
