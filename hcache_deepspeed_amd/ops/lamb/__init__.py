"""``deepspeed.ops.lamb`` import path (reference deepspeed/ops/lamb/__init__.py)."""
from ..optimizers import FusedLamb  # noqa: F401
