"""``deepspeed.ops.adam`` import path (reference deepspeed/ops/adam/__init__.py)."""
from ..cpu_optimizers import DeepSpeedCPUAdam  # noqa: F401
from ..optimizers import FusedAdam  # noqa: F401
