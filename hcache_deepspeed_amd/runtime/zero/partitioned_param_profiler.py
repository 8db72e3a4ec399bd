"""Reference import path (runtime/zero/partitioned_param_profiler.py); implemented in ``comm_stats``."""
from .comm_stats import UnitEventProfiler as PartitionedParameterProfiler  # noqa: F401
