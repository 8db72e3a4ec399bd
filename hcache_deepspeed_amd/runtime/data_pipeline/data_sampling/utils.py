"""Helpers of the data-sampling tools (reference data_sampling/utils.py)."""
import numpy as np


def find_fit_int_dtype(min_value, max_value):
    """Smallest numpy integer dtype holding [min_value, max_value]."""
    if min_value >= 0:
        for dt in (np.uint8, np.uint16, np.uint32, np.uint64):
            if max_value <= np.iinfo(dt).max:
                return dt
    for dt in (np.int8, np.int16, np.int32, np.int64):
        if np.iinfo(dt).min <= min_value and max_value <= np.iinfo(dt).max:
            return dt
    raise ValueError(f"no integer dtype holds [{min_value}, {max_value}]")


def split_index(start_idx, end_idx, num_partitions):
    """[start, end) split into num_partitions contiguous near-equal ranges."""
    n = end_idx - start_idx
    bounds = [start_idx + (n * i) // num_partitions for i in range(num_partitions + 1)]
    return [(bounds[i], bounds[i + 1]) for i in range(num_partitions)]


def split_dataset(dataset, num_workers, worker_id, num_threads):
    lo, hi = split_index(0, len(dataset), num_workers)[worker_id]
    return (lo, hi), split_index(lo, hi, num_threads)
