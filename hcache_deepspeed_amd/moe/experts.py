"""``deepspeed.moe.experts`` import path (reference deepspeed/moe/experts.py)."""
from ..parallel.moe import Experts  # noqa: F401
