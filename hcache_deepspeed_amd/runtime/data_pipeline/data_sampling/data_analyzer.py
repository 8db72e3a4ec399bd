"""Offline data analysis for curriculum learning / data sampling (map-reduce over a dataset).

Reference parity: deepspeed/runtime/data_pipeline/data_sampling/data_analyzer.py ``DataAnalyzer`` :22 (worker x
thread map, multi-process reduce) and ``DistributedDataAnalyzer`` :455 (all ranks map, collective reduce). Output
files (indexed datasets, indexed_dataset.py) and their names are the reference's, so the curriculum sampler of
either framework consumes them:

  ``<save>/<metric>/<metric>_sample_to_metric``                 one item per sample: its value
  ``<save>/<metric>/<metric>_index_to_metric``                  one item per distinct value (ascending)
  ``<save>/<metric>/<metric>_index_to_sample``                  for each distinct value: its sample ids
  ``<save>/<metric>/<metric>_index_to_sample_percentile_merged`` those lists merged into ~100 buckets
  ``<save>/<metric>/<metric>_metric_value``                     accumulate_value_over_samples metrics

Design: the map phase is vectorised -- each (worker, thread) range is read in batches, metric functions run on
whole batches, and a thread's results are kept as numpy arrays (written once, as ``.npy`` partials) instead of
per-sample python dict updates; the reduce is one stable argsort over all samples per metric.
"""
import concurrent.futures as cf
import os

import numpy as np
import torch

from .indexed_dataset import MMapIndexedDataset, close_mmap_dataset_builder, create_mmap_dataset_builder
from .utils import find_fit_int_dtype, split_index

SINGLE = "single_value_per_sample"
ACCUM = "accumulate_value_over_samples"


def _to_numpy(v):
    if torch.is_tensor(v):
        return v.detach().cpu().numpy()
    return np.asarray(v)


def _np(dtype):
    if isinstance(dtype, torch.dtype):
        return torch.empty(0, dtype=dtype).numpy().dtype
    return np.dtype(dtype)


def write_metric_outputs(save_path, name, values, sample_ids, dtype, total_samples=None):
    """Final files of one single_value_per_sample metric from all (value, sample id) pairs."""
    d = os.path.join(save_path, name)
    os.makedirs(d, exist_ok=True)
    values = np.asarray(values).reshape(-1)
    sample_ids = np.asarray(sample_ids, dtype=np.int64).reshape(-1)
    n = int(total_samples if total_samples is not None else (sample_ids.max() + 1 if sample_ids.size else 0))
    sid_dtype = find_fit_int_dtype(0, max(n - 1, 0))
    vdt = _np(dtype)
    # sample -> metric, in sample order
    per_sample = np.zeros(n, dtype=vdt)
    per_sample[sample_ids] = values.astype(vdt)
    b = create_mmap_dataset_builder(os.path.join(d, f"{name}_sample_to_metric"), vdt)
    for v in per_sample:
        b.add_item_numpy(np.array([v], dtype=vdt))
    close_mmap_dataset_builder(b, os.path.join(d, f"{name}_sample_to_metric"))
    # value -> samples
    order = np.lexsort((sample_ids, values))
    sv, ss = values[order], sample_ids[order]
    uniq, starts = np.unique(sv, return_index=True)
    bounds = list(starts) + [len(sv)]
    bi = create_mmap_dataset_builder(os.path.join(d, f"{name}_index_to_sample"), sid_dtype)
    bm = create_mmap_dataset_builder(os.path.join(d, f"{name}_index_to_metric"), vdt)
    for i, u in enumerate(uniq):
        bi.add_item_numpy(ss[bounds[i]:bounds[i + 1]])
        bm.add_item_numpy(np.array([u], dtype=vdt))
    close_mmap_dataset_builder(bi, os.path.join(d, f"{name}_index_to_sample"))
    close_mmap_dataset_builder(bm, os.path.join(d, f"{name}_index_to_metric"))
    # percentile-merged buckets of consecutive distinct values
    step = max(1, len(uniq) // 100)
    bp = create_mmap_dataset_builder(os.path.join(d, f"{name}_index_to_sample_percentile_merged"), sid_dtype)
    for i in range(0, len(uniq), step):
        bp.add_item_numpy(ss[bounds[i]:bounds[min(len(uniq), i + step)]])
    close_mmap_dataset_builder(bp, os.path.join(d, f"{name}_index_to_sample_percentile_merged"))
    return {u.item(): bounds[i + 1] - bounds[i] for i, u in enumerate(uniq)}


def write_accumulated(save_path, name, value, dtype):
    d = os.path.join(save_path, name)
    os.makedirs(d, exist_ok=True)
    fn = os.path.join(d, f"{name}_metric_value")
    b = create_mmap_dataset_builder(fn, _np(dtype))
    b.add_item_numpy(np.asarray(value).reshape(-1))
    close_mmap_dataset_builder(b, fn)


def metric_value_percentiles(num_sample_per_value, step=5):
    """{percentile: metric value} every ``step`` percent (reference get_metric_value_percentiles)."""
    total = sum(num_sample_per_value.values())
    out, seen, cur = {}, 0, step
    for k in sorted(num_sample_per_value):
        seen += num_sample_per_value[k]
        while cur <= 100 and seen >= total * cur / 100.0:
            out[cur] = k
            cur += step
    return out


class DataAnalyzer:

    def __init__(self, dataset, num_workers=1, worker_id=0, num_threads=1, num_threads_reduce=1, specific_threads=(),
                 batch_size=1, metric_names=(), metric_functions=(), metric_types=(), metric_dtypes=(),
                 save_path="./", collate_fn=None, custom_map_init=None, custom_map_update=None,
                 custom_map_finalize=None, custom_reduce=None, sample_indices=None):
        assert len(metric_names) == len(metric_functions) == len(metric_types) == len(metric_dtypes)
        for t in metric_types:
            assert t in (SINGLE, ACCUM), f"unknown metric type {t}"
        self.dataset = dataset
        self.num_workers, self.worker_id = num_workers, worker_id
        self.num_threads, self.num_threads_reduce = num_threads, num_threads_reduce
        self.specific_threads = list(specific_threads)
        self.batch_size = batch_size
        self.metric_names, self.metric_functions = list(metric_names), list(metric_functions)
        self.metric_types, self.metric_dtypes = list(metric_types), list(metric_dtypes)
        self.save_path = save_path
        self.collate_fn = collate_fn
        self.custom_map_init, self.custom_map_update = custom_map_init, custom_map_update
        self.custom_map_finalize, self.custom_reduce = custom_map_finalize, custom_reduce
        self.sample_indices = sample_indices

    # ---- map ------------------------------------------------------------------------------------
    def _partial_dir(self, name, worker, thread):
        return os.path.join(self.save_path, name, f"worker{worker}_thread{thread}")

    def _batches(self, lo, hi):
        for s in range(lo, hi, self.batch_size):
            items = [self.dataset[i] for i in range(s, min(hi, s + self.batch_size))]
            if self.collate_fn is not None:
                yield s, self.collate_fn(items)
            elif torch.is_tensor(items[0]):
                try:
                    yield s, torch.stack(items)
                except RuntimeError:  # ragged samples: the metric functions get the list
                    yield s, items
            else:
                yield s, items

    def _sample_ids(self, data, start, n):
        if isinstance(data, dict) and "index" in data:  # Megatron-style batches carry their sample ids
            return _to_numpy(data["index"]).reshape(n, -1)[:, 0].astype(np.int64)
        ids = np.arange(start, start + n, dtype=np.int64)
        if self.sample_indices is not None:
            ids = np.asarray(self.sample_indices, dtype=np.int64)[ids]
        return ids

    def run_map_helper(self, thread_id):
        (lo, hi) = split_index(0, len(self.dataset), self.num_workers)[self.worker_id]
        tlo, thi = split_index(lo, hi, self.num_threads)[thread_id]
        if self.custom_map_init is not None:
            state = self.custom_map_init(thread_id, self.metric_names, self.metric_types, self.metric_dtypes,
                                         self.save_path, self.worker_id)
        values = [[] for _ in self.metric_names]
        ids = [[] for _ in self.metric_names]
        acc = [None for _ in self.metric_names]
        for start, data in self._batches(tlo, thi):
            if self.custom_map_update is not None:
                self.custom_map_update(data, self.metric_types, self.metric_dtypes, self.metric_functions, state,
                                       start)
                continue
            for m, (fn, mtype, dt) in enumerate(zip(self.metric_functions, self.metric_types, self.metric_dtypes)):
                v = _to_numpy(fn(data))
                if v.dtype != _np(dt):
                    raise TypeError(f"metric {self.metric_names[m]}: function returned {v.dtype}, declared {dt}")
                if mtype == SINGLE:
                    v = v.reshape(v.shape[0], -1)[:, 0]
                    values[m].append(v)
                    ids[m].append(self._sample_ids(data, start, v.shape[0]))
                else:
                    acc[m] = v.copy() if acc[m] is None else acc[m] + v
        if self.custom_map_finalize is not None:
            self.custom_map_finalize(self.metric_types, self.metric_dtypes, state)
            return
        for m, name in enumerate(self.metric_names):
            d = self._partial_dir(name, self.worker_id, thread_id)
            os.makedirs(d, exist_ok=True)
            if self.metric_types[m] == SINGLE:
                v = np.concatenate(values[m]) if values[m] else np.zeros(0, dtype=_np(self.metric_dtypes[m]))
                s = np.concatenate(ids[m]) if ids[m] else np.zeros(0, dtype=np.int64)
                np.save(os.path.join(d, "values.npy"), v)
                np.save(os.path.join(d, "sample_ids.npy"), s)
            elif acc[m] is not None:
                np.save(os.path.join(d, "accumulated.npy"), acc[m])

    def run_map(self):
        threads = self.specific_threads or list(range(self.num_threads))
        if len(threads) == 1:
            self.run_map_helper(threads[0])
            return
        with cf.ThreadPoolExecutor(len(threads)) as ex:
            for f in [ex.submit(self.run_map_helper, t) for t in threads]:
                f.result()

    # ---- reduce -----------------------------------------------------------------------------------
    def _gather_partials(self, name):
        vals, ids, acc = [], [], None
        for w in range(self.num_workers):
            for t in range(self.num_threads):
                d = self._partial_dir(name, w, t)
                if os.path.exists(os.path.join(d, "values.npy")):
                    vals.append(np.load(os.path.join(d, "values.npy")))
                    ids.append(np.load(os.path.join(d, "sample_ids.npy")))
                if os.path.exists(os.path.join(d, "accumulated.npy")):
                    a = np.load(os.path.join(d, "accumulated.npy"))
                    acc = a if acc is None else acc + a
        return vals, ids, acc

    def run_reduce(self):
        if self.custom_reduce is not None:
            self.custom_reduce(self.dataset, self.metric_names, self.metric_types, self.save_path, self.num_workers,
                               self.num_threads, self.num_threads_reduce)
            return
        self.value_percentiles = {}
        for name, mtype, dt in zip(self.metric_names, self.metric_types, self.metric_dtypes):
            vals, ids, acc = self._gather_partials(name)
            if mtype == SINGLE:
                v = np.concatenate(vals) if vals else np.zeros(0, dtype=_np(dt))
                s = np.concatenate(ids) if ids else np.zeros(0, dtype=np.int64)
                counts = write_metric_outputs(self.save_path, name, v, s, dt, total_samples=len(self.dataset))
                self.value_percentiles[name] = metric_value_percentiles(counts)
            elif acc is not None:
                write_accumulated(self.save_path, name, acc, dt)

    def run_map_reduce(self, comm_group=None):
        self.run_map()
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=comm_group)
        if self.worker_id == 0:
            self.run_reduce()
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=comm_group)


class DistributedDataAnalyzer:
    """Every rank maps its contiguous shard; values are gathered with collectives and rank 0 writes the outputs
    (no partial files)."""

    def __init__(self, dataset, num_workers=None, worker_id=None, batch_size=1, metric_names=(),
                 metric_functions=(), metric_types=(), save_path="./", collate_fn=None, device="cpu",
                 comm_group=None, sample_indices=None, metric_dtypes=None):
        dist = torch.distributed
        self.comm_group = comm_group
        self.num_workers = num_workers if num_workers is not None else (
            dist.get_world_size(comm_group) if dist.is_initialized() else 1)
        self.worker_id = worker_id if worker_id is not None else (dist.get_rank(comm_group)
                                                                  if dist.is_initialized() else 0)
        self.inner = DataAnalyzer(dataset, num_workers=self.num_workers, worker_id=self.worker_id,
                                  batch_size=batch_size, metric_names=metric_names, metric_functions=metric_functions,
                                  metric_types=metric_types,
                                  metric_dtypes=metric_dtypes or [torch.int64] * len(metric_names),
                                  save_path=save_path, collate_fn=collate_fn, sample_indices=sample_indices)
        self.device = device

    def run_map_reduce(self):
        a = self.inner
        dist = torch.distributed
        (lo, hi) = split_index(0, len(a.dataset), self.num_workers)[self.worker_id]
        values = [[] for _ in a.metric_names]
        ids = [[] for _ in a.metric_names]
        acc = [None for _ in a.metric_names]
        for start, data in a._batches(lo, hi):
            for m, (fn, mtype) in enumerate(zip(a.metric_functions, a.metric_types)):
                v = _to_numpy(fn(data))
                if mtype == SINGLE:
                    v = v.reshape(v.shape[0], -1)[:, 0]
                    values[m].append(v)
                    ids[m].append(a._sample_ids(data, start, v.shape[0]))
                else:
                    acc[m] = v.copy() if acc[m] is None else acc[m] + v
        for m, (name, mtype, dt) in enumerate(zip(a.metric_names, a.metric_types, a.metric_dtypes)):
            if mtype == SINGLE:
                local = (np.concatenate(values[m]) if values[m] else np.zeros(0, _np(dt)),
                         np.concatenate(ids[m]) if ids[m] else np.zeros(0, np.int64))
                parts = [local]
                if dist.is_initialized() and self.num_workers > 1:
                    parts = [None] * self.num_workers
                    dist.all_gather_object(parts, local, group=self.comm_group)
                if self.worker_id == 0:
                    write_metric_outputs(a.save_path, name, np.concatenate([p[0] for p in parts]),
                                         np.concatenate([p[1] for p in parts]), dt, total_samples=len(a.dataset))
            else:
                t = torch.as_tensor(acc[m] if acc[m] is not None else 0, dtype=torch.float64)
                if dist.is_initialized() and self.num_workers > 1:
                    dist.all_reduce(t, group=self.comm_group)
                if self.worker_id == 0:
                    write_accumulated(a.save_path, name, t.numpy().astype(_np(dt)), dt)
        if dist.is_initialized() and self.num_workers > 1:
            dist.barrier(group=self.comm_group)


def load_sample_to_metric(save_path, metric_name):
    """Per-sample metric values (numpy) from an analyzer output directory (either framework's)."""
    ds = MMapIndexedDataset(os.path.join(save_path, metric_name, f"{metric_name}_sample_to_metric"))
    return np.concatenate(ds[0:len(ds)]) if len(ds) else np.zeros(0)
