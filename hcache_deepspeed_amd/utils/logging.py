"""Logging helpers (reference: deepspeed/utils/logging.py -- LoggerFactory, log_dist, print_json_dist)."""
import json
import logging
import os
import sys

_FMT = "[%(asctime)s] [%(levelname)s] [hds] %(message)s"


def _make_logger(name="hcache_deepspeed_amd", level=logging.INFO):
    lg = logging.getLogger(name)
    if not lg.handlers:
        h = logging.StreamHandler(stream=sys.stdout)
        h.setFormatter(logging.Formatter(_FMT))
        lg.addHandler(h)
        lg.propagate = False
    lg.setLevel(int(os.environ.get("HDS_LOG_LEVEL", level)))
    return lg


logger = _make_logger()
_warned = set()


def _rank():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:
        pass
    return int(os.environ.get("RANK", 0))


def log_dist(message, ranks=None, level=logging.INFO):
    """Log on the given ranks only (None or [-1] -> all ranks)."""
    r = _rank()
    if ranks is None or -1 in ranks or r in ranks:
        logger.log(level, f"[Rank {r}] {message}")


def print_json_dist(message, ranks=None, path=None):
    r = _rank()
    if ranks is None or -1 in ranks or r in ranks:
        message["rank"] = r
        with open(path, "w") as f:
            json.dump(message, f)
            os.fsync(f.fileno())


def warning_once(msg):
    if msg not in _warned:
        _warned.add(msg)
        logger.warning(msg)


def should_log_le(max_level):
    return logger.getEffectiveLevel() <= logging.getLevelName(max_level.upper())


def get_caller_func(frame=3):
    """Name of the function ``frame`` levels up the stack (reference utils/logging.py get_caller_func)."""
    import sys
    return sys._getframe(frame).f_code.co_name
