"""Elastic batch-size planning: one global batch size that stays valid over many GPU counts.

Reference parity: elasticity/elasticity.py (v0.1 ``_get_compatible_gpus_v01`` :83-120 and v0.2
``_get_compatible_gpus_v02`` :123-190, ``compute_elastic_config`` :233) and elasticity/config.py. The
search is the same: candidate batch sizes are (each micro-batch size and their LCM) scaled by the
largest highly-composite multiplier under ``max_train_batch_size``; the winner has the most valid GPU
counts in [min_gpus, max_gpus] (ties -> larger/smaller batch per ``prefer_larger_batch``). v0.2 plans per
node (``num_gpus_per_node``, model parallel size) and returns the micro-batch for the current world.
"""
import json
import math
import os

from ..utils.logging import logger

ELASTICITY = "elasticity"
LATEST_ELASTICITY_VERSION = 0.2
MINIMUM_DEEPSPEED_VERSION = "0.3.8"
DEEPSPEED_ELASTICITY_CONFIG = "DEEPSPEED_ELASTICITY_CONFIG"

# highly composite numbers (more divisors than any smaller integer) up to 720720
HCN_LIST = [
    1, 2, 4, 6, 12, 24, 36, 48, 60, 120, 180, 240, 360, 720, 840, 1260, 1680, 2520, 5040, 7560, 10080, 15120, 20160,
    25200, 27720, 45360, 50400, 55440, 83160, 110880, 166320, 221760, 277200, 332640, 498960, 554400, 665280, 720720
]


class ElasticityError(Exception):
    pass


class ElasticityConfigError(ElasticityError):
    pass


class ElasticityIncompatibleWorldSize(ElasticityError):
    pass


class ElasticityConfig:

    def __init__(self, d):
        self.enabled = bool(d.get("enabled", False))
        if "max_train_batch_size" not in d and self.enabled:
            raise ElasticityConfigError("elasticity config is missing max_train_batch_size")
        if "micro_batch_sizes" not in d and self.enabled:
            raise ElasticityConfigError("elasticity config is missing micro_batch_sizes")
        self.max_acceptable_batch_size = int(d.get("max_train_batch_size", 2000))
        self.micro_batches = list(d.get("micro_batch_sizes", [2, 4, 6]))
        if not all(isinstance(m, int) and m > 0 for m in self.micro_batches):
            raise ElasticityConfigError(f"micro_batch_sizes must be positive ints: {self.micro_batches}")
        self.min_gpus = int(d.get("min_gpus", 1))
        self.max_gpus = int(d.get("max_gpus", 10000))
        if self.min_gpus < 1 or self.max_gpus < 1 or self.min_gpus > self.max_gpus:
            raise ElasticityConfigError(f"invalid min/max gpus {self.min_gpus}/{self.max_gpus}")
        self.model_parallel_size = int(d.get("model_parallel_size", 1))
        self.num_gpus_per_node = int(d.get("num_gpus_per_node", 1))
        self.min_time = int(d.get("min_time", 0))
        self.version = float(d.get("version", LATEST_ELASTICITY_VERSION))
        self.prefer_larger_batch_size = bool(d.get("prefer_larger_batch", True))
        self.ignore_non_elastic_batch_info = bool(d.get("ignore_non_elastic_batch_info", False))

    def __repr__(self):
        return json.dumps(self.__dict__, sort_keys=True)


def get_candidate_batch_sizes(base_list, max_acceptable_batch_size):
    out = set()
    for base in base_list:
        if base >= max_acceptable_batch_size:
            out.add(base)
            continue
        limit = max_acceptable_batch_size // base
        mult = max(h for h in HCN_LIST if h <= limit)
        out.add(mult * base)
    return sorted(out)


def get_valid_gpus(batch_size, micro_batches, min_valid_gpus, max_valid_gpus):
    valid = set()
    for mb in micro_batches:
        if batch_size % mb:
            continue
        max_gpus = batch_size // mb
        if min_valid_gpus <= max_gpus <= max_valid_gpus:
            valid.add(max_gpus)
        for i in range(max(1, min_valid_gpus), min(max_gpus // 2, max_valid_gpus) + 1):
            if max_gpus % i == 0:
                valid.add(i)
    return sorted(valid)


def get_best_candidates(candidate_batch_sizes, micro_batches, min_gpus, max_gpus, prefer_larger):
    best_n, best_gpus, best_bs = 0, None, int(min(micro_batches))
    for bs in candidate_batch_sizes:
        gpus = get_valid_gpus(bs, micro_batches, min_gpus, max_gpus)
        better = len(gpus) > best_n or (len(gpus) == best_n and ((prefer_larger and bs > best_bs) or
                                                                  (not prefer_larger and bs < best_bs)))
        if better:
            best_n, best_gpus, best_bs = len(gpus), gpus, bs
    return best_bs, best_gpus


def _get_compatible_gpus_v01(micro_batches, max_acceptable_batch_size, min_gpus=None, max_gpus=None,
                             prefer_larger=True):
    min_gpus = min_gpus or 1
    max_gpus = max_gpus or max_acceptable_batch_size // min(micro_batches)
    if any(mb > max_acceptable_batch_size for mb in micro_batches):
        raise ValueError(f"all micro batches must be <= max_acceptable_batch_size {max_acceptable_batch_size}")
    lcm = 1
    for mb in micro_batches:
        lcm = lcm * mb // math.gcd(lcm, mb)
    cands = get_candidate_batch_sizes(list(micro_batches) + [lcm], max_acceptable_batch_size)
    return get_best_candidates(cands, micro_batches, min_gpus, max_gpus, prefer_larger)


def _get_compatible_gpus_v02(micro_batches, max_acceptable_batch_size, current_num_gpus, min_gpus=None,
                             max_gpus=None, prefer_larger=True, num_gpus_per_node=1, model_parallel_size=1):
    if num_gpus_per_node % model_parallel_size:
        raise ElasticityError(f"num_gpus_per_node {num_gpus_per_node} must be divisible by model parallel size "
                              f"{model_parallel_size}")

    def pick_micro(final_bs):
        cand = None
        for mb in micro_batches:
            if final_bs // current_num_gpus % mb == 0:
                if cand is None or (prefer_larger and mb > cand):
                    cand = mb
        return cand

    dp_per_node = num_gpus_per_node // model_parallel_size
    bs, valid_nodes = _get_compatible_gpus_v01(micro_batches, int(max_acceptable_batch_size / dp_per_node),
                                               int(min_gpus / num_gpus_per_node), int(max_gpus / num_gpus_per_node),
                                               prefer_larger=prefer_larger)
    bs = int(bs) * dp_per_node
    valid_dp = [n * dp_per_node for n in valid_nodes]
    if current_num_gpus // model_parallel_size in valid_dp:
        return bs, valid_dp, pick_micro(bs)
    cur_dp = (current_num_gpus / num_gpus_per_node) * dp_per_node
    cands = [math.floor(max_acceptable_batch_size / float(mb * cur_dp)) * mb * cur_dp for mb in micro_batches]
    cand = max(cands) if prefer_larger else min(cands)
    return cand, [int(cur_dp)], pick_micro(cand)


def elasticity_enabled(ds_config):
    return bool(ds_config.get(ELASTICITY, {}).get("enabled", False))


def ensure_immutable_elastic_config(runtime_elastic_config_dict):
    if DEEPSPEED_ELASTICITY_CONFIG not in os.environ:
        logger.warning("DEEPSPEED_ELASTICITY_CONFIG not set: cannot verify the scheduler used the same elastic config")
        return
    sched = ElasticityConfig(json.loads(os.environ[DEEPSPEED_ELASTICITY_CONFIG]))
    run = ElasticityConfig(runtime_elastic_config_dict)
    for attr in ("max_acceptable_batch_size", "micro_batches", "version"):
        if getattr(sched, attr) != getattr(run, attr):
            raise ElasticityConfigError(f"elastic config {attr}: scheduler saw {getattr(sched, attr)}, runtime has "
                                        f"{getattr(run, attr)}")


def _version_tuple(v):
    return tuple(int(x) for x in str(v).split("+")[0].split(".")[:3] if x.isdigit())


def compute_elastic_config(ds_config, target_deepspeed_version, world_size=0, return_microbatch=False):
    """Returns (final_batch_size, valid_gpus[, micro_batch_size])."""
    if not isinstance(ds_config, dict):
        raise ValueError(f"expected a dict config, got {type(ds_config)}")
    if ELASTICITY not in ds_config:
        raise ElasticityConfigError("'elasticity' is missing from the config")
    d = ds_config[ELASTICITY]
    if not d.get("enabled", False):
        raise ElasticityConfigError("elasticity is disabled ('enabled': true to use it)")
    ec = ElasticityConfig(d)
    if ec.model_parallel_size > 1 and ec.version != 0.2:
        raise ElasticityConfigError(f"elasticity v{ec.version} does not support model parallelism")
    if ec.version > LATEST_ELASTICITY_VERSION:
        raise ElasticityConfigError(f"elasticity version {ec.version} > supported {LATEST_ELASTICITY_VERSION}")
    if _version_tuple(target_deepspeed_version) < _version_tuple(MINIMUM_DEEPSPEED_VERSION):
        raise ElasticityError(f"target version {target_deepspeed_version} < {MINIMUM_DEEPSPEED_VERSION}")
    micro = None
    if ec.version == 0.1:
        bs, gpus = _get_compatible_gpus_v01(ec.micro_batches, ec.max_acceptable_batch_size, ec.min_gpus, ec.max_gpus,
                                            ec.prefer_larger_batch_size)
    elif ec.version == 0.2:
        cur = world_size or int(os.environ.get("WORLD_SIZE", "0") or 0)
        if cur <= 0:
            raise ElasticityConfigError("elasticity v0.2 needs world_size (argument or WORLD_SIZE env)")
        bs, gpus, micro = _get_compatible_gpus_v02(ec.micro_batches, ec.max_acceptable_batch_size, cur, ec.min_gpus,
                                                   ec.max_gpus, ec.prefer_larger_batch_size, ec.num_gpus_per_node,
                                                   ec.model_parallel_size)
    else:
        raise NotImplementedError(f"elasticity version {ec.version}")
    bs = int(bs)
    if world_size > 0:
        if world_size not in gpus:
            raise ElasticityIncompatibleWorldSize(f"world size {world_size} not in valid GPU counts {gpus}")
        mbs = next((m for m in sorted(set(ec.micro_batches), reverse=True) if bs // world_size % m == 0), None)
        assert mbs is not None, "no micro batch size divides the per-GPU batch"
        return bs, gpus, mbs
    if return_microbatch:
        return bs, gpus, micro
    return bs, gpus
