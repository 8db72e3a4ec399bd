"""Checkpoint utilities: zero_to_fp32 consolidation and universal (re-shardable) checkpoints."""
from .universal import ds_to_universal, load_universal_into  # noqa: F401
from .zero_to_fp32 import (convert_zero_checkpoint_to_fp32_state_dict,  # noqa: F401
                           get_fp32_state_dict_from_zero_checkpoint, load_state_dict_from_zero_checkpoint)
