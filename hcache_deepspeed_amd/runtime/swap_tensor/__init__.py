"""NVMe tier of ZeRO-Infinity (reference runtime/swap_tensor/: partitioned_param_swapper.py,
partitioned_optimizer_swapper.py, pipelined_optimizer_swapper.py, aio_config.py)."""
from .aio_config import get_aio_config  # noqa: F401
from .partitioned_param_swapper import AsyncPartitionedParameterSwapper  # noqa: F401
from .pipelined_optimizer_swapper import PipelinedOptimizerSwapper  # noqa: F401
