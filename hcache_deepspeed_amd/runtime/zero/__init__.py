"""ZeRO (flat-shard) public surface: ``zero.Init``, ``zero.GatheredParameters`` and the optimizers (reference
runtime/zero/__init__.py: ZeroParamType, ZeroParamStatus, Init, GatheredParameters, register_external_parameter,
TiledLinear, TiledLinearReturnBias, MiCS_Init, unwrap_model_for_generation)."""
import contextlib
import enum

from .flat import ZeroParamStatus  # noqa: F401
from .mics import MiCS_Init  # noqa: F401
from .optimizer import DeepSpeedZeroOptimizer, DeepSpeedZeroOptimizer_Stage3, ZeroOptimizer  # noqa: F401
from .partition_parameters import (GatheredParameters, Init, get_z3_leaf_modules,  # noqa: F401
                                   register_external_parameter, set_z3_leaf_modules, unregister_external_parameter)
from .tiling import TiledLinear, TiledLinearReturnBias  # noqa: F401


class ZeroParamType(enum.Enum):
    # same values as the reference enum: a regular parameter, one partitioned by ZeRO-3, one held remotely (host/NVMe)
    NORMAL = 1
    PARTITIONED = 2
    REMOTE = 3


@contextlib.contextmanager
def unwrap_model_for_generation(model):
    """Yield the bare module for generation, with every ZeRO-3 partition gathered for the duration (reference
    runtime/zero/__init__.py -> utils' unwrap_model_for_generation, used by TRL): generation runs many short
    forwards, which would otherwise all-gather every unit per token."""
    module = getattr(model, "module", model)
    z = getattr(model, "optimizer", None)
    if z is not None and getattr(z, "stage", 0) == 3 and getattr(z, "partitioned", False):
        with GatheredParameters(list(module.parameters())):
            yield module
    else:
        yield module
