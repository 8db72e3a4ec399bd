"""MiCS (Zhang et al., "MiCS: Near-linear Scaling for Training Gigantic Model on Public Cloud"): parameters sharded
over small groups of ``mics_shard_size`` ranks and replicated across the groups.

Reference: runtime/zero/mics.py -- ``MiCS_Init`` (partition at construction over the shard group), the MiCS
optimizer (reduce-scatter inside the shard group + all-reduce across the replicas). The optimizer half lives in the
flat ZeRO optimizer (runtime/zero/optimizer.py ``_setup_zeropp``: shard / replica groups from contiguous rank blocks,
i.e. one xGMI island per shard group on an MI355X node); this module is the construction-time half.
"""
import json
import os

from ... import comm as dist
from .partition_parameters import Init


def _shard_size_from(config_dict_or_path, config):
    cfg = config if config is not None else config_dict_or_path
    if cfg is None:
        return None
    if hasattr(cfg, "zero_config"):
        return int(cfg.zero_config.mics_shard_size)
    if isinstance(cfg, str):
        if os.path.exists(cfg):
            with open(cfg) as f:
                cfg = json.load(f)
        else:
            cfg = json.loads(cfg)
    return int((cfg.get("zero_optimization") or {}).get("mics_shard_size", -1))


def mics_shard_group(shard_size, ranks=None):
    """This rank's shard group: contiguous blocks of ``shard_size`` ranks (every rank creates every block, as
    ``new_group`` requires). Returns (group, block ranks)."""
    ranks = list(ranks) if ranks is not None else list(range(dist.get_world_size()))
    if len(ranks) % shard_size:
        raise ValueError(f"mics_shard_size {shard_size} must divide the data-parallel size {len(ranks)}")
    me, mine = dist.get_rank(), None
    for i in range(0, len(ranks), shard_size):
        block = ranks[i:i + shard_size]
        g = dist.new_group(ranks=block)
        if me in block:
            mine = (g, block)
    return mine


class MiCS_Init(Init):
    """``zero.Init`` whose partitions span only this rank's MiCS shard group (``zero_optimization.mics_shard_size``
    from ``config_dict_or_path`` / ``config``, or ``mics_shard_size``): each parameter is split over shard_size ranks
    instead of the whole data-parallel world, and the optimizer's MiCS layout adopts those partitions."""

    def __init__(self, module=None, data_parallel_group=None, sequence_data_parallel_group=None,
                 mem_efficient_linear=True, remote_device=None, pin_memory=False, config_dict_or_path=None, config=None,
                 enabled=True, dtype=None, mpu=None, mics_shard_size=None, **kw):
        dist.init_distributed(verbose=False)
        size = mics_shard_size if mics_shard_size is not None else _shard_size_from(config_dict_or_path, config)
        if not size or size <= 0:
            raise ValueError("MiCS_Init needs zero_optimization.mics_shard_size > 0")
        self.mics_shard_size = int(size)
        group = None
        if enabled and dist.is_initialized() and dist.get_world_size() > 1:
            base = data_parallel_group or sequence_data_parallel_group
            ranks = dist.get_all_ranks_from_group(base) if base is not None else None
            group, self.mics_ranks = mics_shard_group(self.mics_shard_size, ranks)
        super().__init__(module=module, data_parallel_group=group, mem_efficient_linear=mem_efficient_linear,
                         remote_device=remote_device, pin_memory=pin_memory, config_dict_or_path=config_dict_or_path,
                         config=config, enabled=enabled, dtype=dtype, mpu=mpu, **kw)
