"""``deepspeed.utils.zero_to_fp32`` import path (reference deepspeed/utils/zero_to_fp32.py)."""
from ..checkpoint.zero_to_fp32 import (convert_zero_checkpoint_to_fp32_state_dict,  # noqa: F401
                                       get_fp32_state_dict_from_zero_checkpoint, load_state_dict_from_zero_checkpoint)
