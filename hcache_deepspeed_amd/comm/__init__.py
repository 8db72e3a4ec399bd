"""Collective communication facade (``import hcache_deepspeed_amd.comm as dist``)."""
from .comm import *  # noqa: F401,F403
from .comm import (ReduceOp, all_gather, all_gather_into_tensor, all_reduce, all_to_all_single, barrier, broadcast,
                   configure, get_local_rank, get_rank, get_world_size, init_distributed, is_initialized, log_summary,
                   new_group, reduce_scatter_tensor)
