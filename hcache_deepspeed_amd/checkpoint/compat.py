"""Let ``torch.load(..., weights_only=True)`` read checkpoints the reference DeepSpeed wrote.

The reference pickles a few of its own classes into checkpoint files (the loss scaler object, the
``ZeroStageEnum`` stage value, ``fragment_address`` slice mappings, ``SubparamShape``). A weights-only
load refuses unknown globals, and we never unpickle with ``weights_only=False``; instead each reference
class path is mapped onto this framework's equivalent class, which has the same attributes. Importing
this module registers the mapping (idempotent).
"""
from dataclasses import dataclass
from enum import Enum
from typing import List, Tuple, Union

import torch

from ..runtime.fp16.loss_scaler import DynamicLossScaler, LossScaler
from ..utils.tensor_fragment import fragment_address


class ZeroStageEnum(int, Enum):
    """Reference runtime/zero/config.py:77."""
    disabled = 0
    optimizer_states = 1
    gradients = 2
    weights = 3
    max_stage = 3


@dataclass
class SubparamShape:
    """A fused parameter made of sub-parameters that are TP-partitioned independently (e.g. fused QKV).
    Reference checkpoint/universal_checkpoint.py:15."""
    patterns: List[str]
    shape: Tuple[Union[Tuple[int], int]]
    partition_dim: int


_REF_CLASSES = [
    (fragment_address, "deepspeed.utils.tensor_fragment.fragment_address"),
    (LossScaler, "deepspeed.runtime.fp16.loss_scaler.LossScaler"),
    (DynamicLossScaler, "deepspeed.runtime.fp16.loss_scaler.DynamicLossScaler"),
    (ZeroStageEnum, "deepspeed.runtime.zero.config.ZeroStageEnum"),
    (SubparamShape, "deepspeed.checkpoint.universal_checkpoint.SubparamShape"),
]

torch.serialization.add_safe_globals(_REF_CLASSES + [ZeroStageEnum, SubparamShape, fragment_address])
