"""Static / dynamic loss scaling (reference: runtime/fp16/loss_scaler.py:42,67,91,208).

The overflow flag itself is computed on the GPU (ops/optimizers.grad_sumsq sets a device int and the
fused optimizer kernels skip the update when it is set); the scaler only needs the flag's value once
per optimizer step to update the scale.
"""
INITIAL_LOSS_SCALE = "init_scale"
SCALE_WINDOW = "scale_window"
DELAYED_SHIFT = "delayed_shift"
CONSECUTIVE_HYSTERESIS = "consecutive_hysteresis"
MIN_LOSS_SCALE = "min_scale"


class LossScalerBase:

    def __init__(self, cur_scale):
        self.cur_scale = float(cur_scale)
        self.dynamic = False

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def update_scale(self, overflow):
        pass

    def backward(self, loss, retain_graph=False):
        (loss * self.loss_scale).backward(retain_graph=retain_graph)

    def state_dict(self):
        return {"cur_scale": self.cur_scale}

    def load_state_dict(self, sd):
        self.cur_scale = sd["cur_scale"]


class LossScaler(LossScalerBase):
    """Static loss scale."""

    def has_overflow(self, params):
        return False


class DynamicLossScaler(LossScalerBase):

    def __init__(self, init_scale=2**32, scale_factor=2.0, scale_window=1000, min_scale=1, delayed_shift=1,
                 consecutive_hysteresis=False, raise_error_at_min_scale=True, dtype=None):
        super().__init__(init_scale)
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.delayed_shift = delayed_shift
        self.cur_hysteresis = delayed_shift
        self.consecutive_hysteresis = consecutive_hysteresis
        self.raise_error_at_min_scale = raise_error_at_min_scale
        self.dynamic = True

    def update_scale(self, overflow):
        if overflow:
            if self.delayed_shift == 1 or self.cur_hysteresis == 1:
                if self.cur_scale == self.min_scale and self.raise_error_at_min_scale:
                    raise Exception("Current loss scale already at minimum - cannot decrease scale anymore.")
                self.cur_scale = max(self.cur_scale / self.scale_factor, self.min_scale)
            else:
                self.cur_hysteresis -= 1
            self.last_overflow_iter = self.cur_iter
        else:
            if self.consecutive_hysteresis:
                self.cur_hysteresis = self.delayed_shift
            if (self.cur_iter - self.last_overflow_iter) % self.scale_window == 0:
                if not self.consecutive_hysteresis:
                    self.cur_hysteresis = self.delayed_shift
                self.cur_scale *= self.scale_factor
        self.cur_iter += 1

    def state_dict(self):
        return {"cur_scale": self.cur_scale, "cur_iter": self.cur_iter, "last_overflow_iter": self.last_overflow_iter,
                "cur_hysteresis": self.cur_hysteresis}

    def load_state_dict(self, sd):
        for k, v in sd.items():
            setattr(self, k, v)


def CreateLossScaler(dtype, static_loss_scale, dynamic_scaling, dynamic_loss_args):
    import torch
    if dtype == torch.float16 and dynamic_scaling:
        args = dynamic_loss_args or {}
        return DynamicLossScaler(init_scale=args.get(INITIAL_LOSS_SCALE, 2**16),
                                 scale_window=args.get(SCALE_WINDOW, 1000), min_scale=args.get(MIN_LOSS_SCALE, 1),
                                 delayed_shift=args.get(DELAYED_SHIFT, 2),
                                 consecutive_hysteresis=args.get(CONSECUTIVE_HYSTERESIS, False))
    scale = static_loss_scale if dtype == torch.float16 else 1.0
    return LossScaler(scale)
