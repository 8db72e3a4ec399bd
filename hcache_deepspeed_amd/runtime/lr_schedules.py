"""LR schedules with the reference names and config keys (runtime/lr_schedules.py:273,371,633,723,774)."""
import math

LR_RANGE_TEST, ONE_CYCLE, WARMUP_LR, WARMUP_DECAY_LR, WARMUP_COSINE_LR = ("LRRangeTest", "OneCycle", "WarmupLR",
                                                                        "WarmupDecayLR", "WarmupCosineLR")
VALID_LR_SCHEDULES = [LR_RANGE_TEST, ONE_CYCLE, WARMUP_LR, WARMUP_DECAY_LR, WARMUP_COSINE_LR]


class _Sched:

    def __init__(self, optimizer, last_batch_iteration=-1):
        self.optimizer = optimizer
        self.last_batch_iteration = last_batch_iteration
        self._last_lr = None

    def get_lr(self):
        raise NotImplementedError

    def get_last_lr(self):
        return self._last_lr

    def step(self, last_batch_iteration=None):
        if last_batch_iteration is None:
            last_batch_iteration = self.last_batch_iteration + 1
        self.last_batch_iteration = last_batch_iteration
        lrs = self.get_lr()
        for g, lr in zip(self.optimizer.param_groups, lrs):
            g["lr"] = lr
        self._last_lr = [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd):
        self.last_batch_iteration = sd["last_batch_iteration"]


class WarmupLR(_Sched):

    def __init__(self, optimizer, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 warmup_type="log", last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        n = len(optimizer.param_groups)
        self.min_lrs = warmup_min_lr if isinstance(warmup_min_lr, (list, tuple)) else [warmup_min_lr] * n
        self.max_lrs = warmup_max_lr if isinstance(warmup_max_lr, (list, tuple)) else [warmup_max_lr] * n
        self.delta_lrs = [b - a for a, b in zip(self.min_lrs, self.max_lrs)]
        self.warmup_num_steps = max(2, warmup_num_steps)
        self.warmup_type = warmup_type
        self.inverse_log_warm_up = 1.0 / math.log(self.warmup_num_steps)
        if last_batch_iteration == -1:
            self._last_lr = [g.get("lr") for g in optimizer.param_groups]

    def _gamma(self):
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            if self.warmup_type == "log":
                return self.inverse_log_warm_up * math.log(it + 1)
            return it / self.warmup_num_steps
        return 1.0

    def get_lr(self):
        if self.last_batch_iteration < 0:
            return [0.0 for _ in self.min_lrs]
        g = self._gamma()
        return [a + d * g for a, d in zip(self.min_lrs, self.delta_lrs)]


class WarmupDecayLR(WarmupLR):

    def __init__(self, optimizer, total_num_steps, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 warmup_type="log", last_batch_iteration=-1):
        self.total_num_steps = total_num_steps
        super().__init__(optimizer, warmup_min_lr, warmup_max_lr, warmup_num_steps, warmup_type, last_batch_iteration)

    def _gamma(self):
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            return super()._gamma()
        return max(0.0, (self.total_num_steps - it) / max(1.0, self.total_num_steps - self.warmup_num_steps))


class WarmupCosineLR(_Sched):

    def __init__(self, optimizer, total_num_steps, warmup_min_ratio=0.0, warmup_num_steps=1000, cos_min_ratio=0.0001,
                 warmup_type="log", last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        self.total_num_steps = total_num_steps
        self.warmup_min_ratio = warmup_min_ratio
        self.warmup_num_steps = max(2, warmup_num_steps)
        self.cos_min_ratio = cos_min_ratio
        self.warmup_type = warmup_type
        self.org_lrs = [g["lr"] for g in optimizer.param_groups]
        self.inverse_log_warm_up = 1.0 / math.log(self.warmup_num_steps)

    def get_lr_ratio(self):
        it = self.last_batch_iteration
        if it < 0:
            return 0.0
        if it < self.warmup_num_steps:
            if self.warmup_type == "log":
                r = self.inverse_log_warm_up * math.log(it + 1)
            else:
                r = it / self.warmup_num_steps
            return self.warmup_min_ratio + (1.0 - self.warmup_min_ratio) * r
        ratio_delta = 1.0 - self.cos_min_ratio
        frac = (it - self.warmup_num_steps) / max(1, self.total_num_steps - self.warmup_num_steps)
        frac = min(1.0, frac)
        return self.cos_min_ratio + ratio_delta * 0.5 * (1 + math.cos(math.pi * frac))

    def get_lr(self):
        r = self.get_lr_ratio()
        return [lr * r for lr in self.org_lrs]


class OneCycle(_Sched):

    def __init__(self, optimizer, cycle_min_lr, cycle_max_lr, decay_lr_rate=0.0, cycle_first_step_size=2000,
                 cycle_second_step_size=None, cycle_first_stair_count=0, cycle_second_stair_count=None,
                 decay_step_size=0, cycle_momentum=True, cycle_min_mom=0.8, cycle_max_mom=0.9, decay_mom_rate=0.0,
                 last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        self.min_lr, self.max_lr = cycle_min_lr, cycle_max_lr
        self.first = cycle_first_step_size
        self.second = cycle_second_step_size if cycle_second_step_size is not None else cycle_first_step_size
        self.total = self.first + self.second
        self.decay_lr_rate = decay_lr_rate
        self.decay_step_size = decay_step_size

    def get_lr(self):
        it = max(0, self.last_batch_iteration)
        if it <= self.total:
            if it <= self.first:
                f = it / self.first
            else:
                f = 1 - (it - self.first) / self.second
            lr = self.min_lr + (self.max_lr - self.min_lr) * f
        else:
            decay = (it - self.total) / self.decay_step_size if self.decay_step_size else 0
            lr = self.min_lr / (1 + self.decay_lr_rate * decay)
        return [lr for _ in self.optimizer.param_groups]


class LRRangeTest(_Sched):

    def __init__(self, optimizer, lr_range_test_min_lr=1e-3, lr_range_test_step_size=2000,
                 lr_range_test_step_rate=1.0, lr_range_test_staircase=False, last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        self.min_lr = lr_range_test_min_lr
        self.step_size = lr_range_test_step_size
        self.step_rate = lr_range_test_step_rate
        self.staircase = lr_range_test_staircase

    def get_lr(self):
        it = max(0, self.last_batch_iteration)
        x = it / self.step_size
        if self.staircase:
            x = math.floor(x)
        return [self.min_lr * (1 + x * self.step_rate) for _ in self.optimizer.param_groups]


def get_scheduler(name, optimizer, params):
    cls = {LR_RANGE_TEST: LRRangeTest, ONE_CYCLE: OneCycle, WARMUP_LR: WarmupLR, WARMUP_DECAY_LR: WarmupDecayLR,
           WARMUP_COSINE_LR: WarmupCosineLR}.get(name)
    if cls is None:
        import torch
        cls = getattr(torch.optim.lr_scheduler, name)
    return cls(optimizer, **params)


def add_tuning_arguments(parser):
    """LR-schedule command-line arguments (reference runtime/lr_schedules.py add_tuning_arguments)."""
    g = parser.add_argument_group("Convergence Tuning", "Convergence tuning configurations")
    g.add_argument("--lr_schedule", type=str, default=None, help="LR schedule for training.")
    g.add_argument("--lr_range_test_min_lr", type=float, default=0.001)
    g.add_argument("--lr_range_test_step_rate", type=float, default=1.0)
    g.add_argument("--lr_range_test_step_size", type=int, default=1000)
    g.add_argument("--lr_range_test_staircase", type=bool, default=False)
    g.add_argument("--cycle_first_step_size", type=int, default=1000)
    g.add_argument("--cycle_first_stair_count", type=int, default=-1)
    g.add_argument("--cycle_second_step_size", type=int, default=-1)
    g.add_argument("--cycle_second_stair_count", type=int, default=-1)
    g.add_argument("--decay_step_size", type=int, default=1000)
    g.add_argument("--cycle_min_lr", type=float, default=0.01)
    g.add_argument("--cycle_max_lr", type=float, default=0.1)
    g.add_argument("--decay_lr_rate", type=float, default=0.0)
    g.add_argument("--cycle_momentum", default=False, action="store_true")
    g.add_argument("--cycle_min_mom", type=float, default=0.8)
    g.add_argument("--cycle_max_mom", type=float, default=0.9)
    g.add_argument("--decay_mom_rate", type=float, default=0.0)
    g.add_argument("--warmup_min_lr", type=float, default=0)
    g.add_argument("--warmup_max_lr", type=float, default=0.001)
    g.add_argument("--warmup_num_steps", type=int, default=1000)
    g.add_argument("--warmup_type", type=str, default="log")
    g.add_argument("--warmup_min_ratio", type=float, default=0.0)
    g.add_argument("--cos_min_ratio", type=float, default=0.0001)
    return parser
