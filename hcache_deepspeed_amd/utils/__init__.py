"""Utilities: logging, timers, process groups, NUMA binding, and the tensor-fragment (safe_get_*) APIs."""
from .logging import logger, log_dist  # noqa: F401
from .tensor_fragment import (safe_get_full_fp32_param, safe_get_full_grad, safe_get_full_optimizer_state,  # noqa
                              safe_get_local_fp32_param, safe_get_local_grad, safe_get_local_optimizer_state,
                              safe_set_full_fp32_param, safe_set_full_grad, safe_set_full_optimizer_state,
                              safe_set_local_fp32_param, safe_set_local_grad, safe_set_local_optimizer_state)
from .tensor_fragment import fragment_address  # noqa: F401
from .init_on_device import OnDevice  # noqa: F401
from .nvtx import instrument_w_nvtx  # noqa: F401
from .numa import get_numactl_cmd  # noqa: F401
from ..runtime.zero.partition_parameters import get_z3_leaf_modules, set_z3_leaf_modules  # noqa: F401
