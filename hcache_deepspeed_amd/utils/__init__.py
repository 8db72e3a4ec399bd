"""Utilities: logging, timers, process groups, NUMA binding, and the tensor-fragment (safe_get_*) APIs."""
from .logging import logger, log_dist  # noqa: F401
from .tensor_fragment import (safe_get_full_fp32_param, safe_get_full_grad, safe_get_full_optimizer_state,  # noqa
                              safe_get_local_fp32_param, safe_get_local_grad, safe_get_local_optimizer_state,
                              safe_set_full_fp32_param, safe_set_full_grad, safe_set_full_optimizer_state,
                              safe_set_local_fp32_param, safe_set_local_grad, safe_set_local_optimizer_state)
from .tensor_fragment import fragment_address  # noqa: F401
from .tensor_fragment import (get_full_hp_grad, get_full_hp_param, get_hp_fragment_mapping,  # noqa: F401
                              lazy_init_hp_params_optimizer_state, link_hp_params, map_to_flat_opt_states,
                              set_full_hp_grad, set_full_hp_param)
from . import tensor_fragment  # noqa: F401
from .logging import get_caller_func  # noqa: F401
from .init_on_device import OnDevice  # noqa: F401
from .nvtx import instrument_w_nvtx  # noqa: F401
from .numa import get_numactl_cmd  # noqa: F401
from ..runtime.zero.partition_parameters import (get_z3_leaf_modules, set_z3_leaf_module,  # noqa: F401
                                                 set_z3_leaf_modules, unset_z3_leaf_modules, z3_leaf_module,
                                                 z3_leaf_parameter)
from ..runtime.dataloader import RepeatingLoader  # noqa: F401
