"""Reference import path (deepspeed/runtime/bf16_optimizer.py); implementation in runtime/fp16/fused_optimizer.py."""
from .fp16.fused_optimizer import BF16_Optimizer  # noqa: F401
