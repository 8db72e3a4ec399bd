"""``deepspeed.moe.utils`` import path (reference deepspeed/moe/utils.py)."""
from ..parallel.moe import is_moe_param, split_params_into_different_moe_groups_for_optimizer  # noqa: F401
