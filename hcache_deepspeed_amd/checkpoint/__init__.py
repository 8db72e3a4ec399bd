"""Checkpoint utilities: zero_to_fp32 consolidation and universal (re-shardable) checkpoints, both on the
reference's on-disk schema (constants.py)."""
from . import compat  # noqa: F401
from .constants import *  # noqa: F401,F403
from .compat import SubparamShape  # noqa: F401
from .universal import ds_to_universal, load_universal_into  # noqa: F401
from .zero_to_fp32 import (convert_zero_checkpoint_to_fp32_state_dict,  # noqa: F401
                           get_fp32_state_dict_from_zero_checkpoint, load_state_dict_from_zero_checkpoint)
