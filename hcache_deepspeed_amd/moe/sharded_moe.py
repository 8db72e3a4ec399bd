"""``deepspeed.moe.sharded_moe`` import path (reference deepspeed/moe/sharded_moe.py)."""
from ..parallel.moe import MOELayer, TopKGate  # noqa: F401
