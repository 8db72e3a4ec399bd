"""``aio`` config section (reference runtime/swap_tensor/aio_config.py, constants.py)."""

AIO_DEFAULTS = {
    "block_size": 1 << 20,
    "queue_depth": 32,
    "intra_op_parallelism": 4,
    "single_submit": False,
    "overlap_events": True,
    "use_gds": False,
}


def get_aio_config(d):
    cfg = dict(AIO_DEFAULTS)
    cfg.update({k: v for k, v in (d or {}).items() if k in AIO_DEFAULTS or k == "thread_count"})
    if "thread_count" in cfg:  # older key name
        cfg["intra_op_parallelism"] = cfg.pop("thread_count")
    return cfg


def make_aio_handle(d):
    from ...ops.aio import aio_handle
    c = get_aio_config(d)
    return aio_handle(c["block_size"], c["queue_depth"], c["single_submit"], c["overlap_events"],
                      c["intra_op_parallelism"])
