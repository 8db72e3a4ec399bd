"""``deepspeed.ops.lion`` import path (reference deepspeed/ops/lion/__init__.py)."""
from ..cpu_optimizers import DeepSpeedCPULion  # noqa: F401
from ..optimizers import FusedLion  # noqa: F401
