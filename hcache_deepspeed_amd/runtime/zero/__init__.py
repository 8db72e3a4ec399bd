"""ZeRO (flat-shard) public surface: ``zero.Init``, ``zero.GatheredParameters`` and the optimizers."""
from .flat import ZeroParamStatus  # noqa: F401
from .optimizer import DeepSpeedZeroOptimizer, DeepSpeedZeroOptimizer_Stage3, ZeroOptimizer  # noqa: F401
from .partition_parameters import (GatheredParameters, Init, get_z3_leaf_modules,  # noqa: F401
                                   register_external_parameter, set_z3_leaf_modules, unregister_external_parameter)
