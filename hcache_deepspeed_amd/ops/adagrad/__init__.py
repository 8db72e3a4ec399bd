"""``deepspeed.ops.adagrad`` import path (reference deepspeed/ops/adagrad/__init__.py)."""
from ..cpu_optimizers import DeepSpeedCPUAdagrad  # noqa: F401
