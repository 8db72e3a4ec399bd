"""``deepspeed.moe.layer`` import path (reference deepspeed/moe/layer.py:17)."""
from ..parallel.moe import MoE  # noqa: F401
