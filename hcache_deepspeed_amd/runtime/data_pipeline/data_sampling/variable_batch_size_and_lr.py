"""Variable batch size by token budget, with the learning rate scaled to each batch's size.

Reference parity: deepspeed/runtime/data_pipeline/data_sampling/variable_batch_size_and_lr.py (``batch_by_seqlens``
:23, ``scale_lr`` :149, ``dataloader_for_variable_batch_size`` :165, ``VariableBatchSizeLR`` :226,
``lr_scheduler_for_variable_batch_size`` :308, ``get_dataloader_and_lr_scheduler_for_variable_batch_size`` :432).

Packing is a single greedy pass over the samples in the chosen order: a micro-batch closes when the next sample
would exceed ``max_tokens`` (or ``max_batch_size``), and ``effective_batch_size`` consecutive micro-batches form one
optimizer batch (one per data-parallel rank x gradient-accumulation step).
"""
import math
import random

import numpy as np
import torch
from torch.utils.data import DataLoader, DistributedSampler


def batch_by_seqlens(seqlens, max_tokens, sequence_ids_per_mb=None, min_batch_size=1, max_batch_size=None,
                     sequence_picking_order="dataloader", effective_batch_size=1,
                     required_microbatches_of_same_size=False, verbose=False, seed=None):
    """Returns (microbatch_ids [(batch_id, [sample ids])], batch_sizes [samples per batch], batch_max_seqlens)."""
    assert sequence_picking_order in ("random", "seqlen", "dataloader")
    seqlens = np.asarray(seqlens)
    ids = np.arange(len(seqlens)) if sequence_ids_per_mb is None else np.asarray(sequence_ids_per_mb)
    order = list(ids)
    if sequence_picking_order == "random":
        random.Random(seed).shuffle(order)
    elif sequence_picking_order == "seqlen":
        order = sorted(order, key=lambda i: (seqlens[i], i))
    order = [i for i in order if seqlens[i] <= max_tokens]  # a sample alone over the budget cannot be placed
    mbs, cur, cur_tok = [], [], 0
    for i in order:
        full = (max_batch_size is not None and len(cur) >= max_batch_size)
        if cur and (cur_tok + seqlens[i] > max_tokens or full):
            mbs.append(cur)
            cur, cur_tok = [], 0
        cur.append(int(i))
        cur_tok += int(seqlens[i])
    if cur:
        mbs.append(cur)
    mbs = [m for m in mbs if len(m) >= min_batch_size]
    n_batches = len(mbs) // effective_batch_size
    mbs = mbs[:n_batches * effective_batch_size]
    if required_microbatches_of_same_size:
        # every micro-batch of a batch gets the batch's smallest micro-batch size (surplus samples dropped)
        for b in range(n_batches):
            grp = mbs[b * effective_batch_size:(b + 1) * effective_batch_size]
            k = min(len(m) for m in grp)
            for j in range(len(grp)):
                mbs[b * effective_batch_size + j] = grp[j][:k]
    microbatch_ids, batch_sizes, batch_max_seqlens = [], [], []
    for b in range(n_batches):
        grp = mbs[b * effective_batch_size:(b + 1) * effective_batch_size]
        microbatch_ids.extend((b, m) for m in grp)
        batch_sizes.append(sum(len(m) for m in grp))
        batch_max_seqlens.append(int(max(seqlens[i] for m in grp for i in m)))
    if verbose:
        print(f"batch_by_seqlens: {len(microbatch_ids)} micro-batches in {n_batches} batches, "
              f"sizes {min(batch_sizes, default=0)}..{max(batch_sizes, default=0)}")
    return microbatch_ids, batch_sizes, batch_max_seqlens


def scale_lr(base_batch_size, batch_size, base_lr=1, method="linear"):
    if method == "linear":
        return base_lr * batch_size / base_batch_size
    if method == "sqrt":
        return base_lr * math.sqrt(batch_size / base_batch_size)
    if method is None or str(method).upper() == "NONE":
        return base_lr
    raise ValueError(f"unknown LR scaling method {method!r}")


def dataloader_for_variable_batch_size(dataset, microbatch_ids, batch_max_seqlens, dataloader_rank=0,
                                       dataloader_batch_size=1, dataloader_num_replicas=1, dataloader_collate_fn=None,
                                       dataloader_num_workers=2, dataloader_pin_memory=False,
                                       required_microbatches_of_same_seqlen=False, sample_padding_fn=None):
    """Micro-batches are dealt to the data-parallel replicas round-robin; each loader item is one micro-batch."""
    sampler = DistributedSampler(microbatch_ids, num_replicas=dataloader_num_replicas, rank=dataloader_rank,
                                 shuffle=False, drop_last=False)

    def collate(list_microbatch_ids):
        batch = []
        for batch_id, ids in list_microbatch_ids:
            samples = [dataset[i] for i in ids]
            if required_microbatches_of_same_seqlen:
                assert sample_padding_fn is not None, "sample_padding_fn is required to pad to the batch max seqlen"
                L = batch_max_seqlens[batch_id]
                samples = [sample_padding_fn(s, L) for s in samples]
            batch += samples
        return dataloader_collate_fn(batch) if dataloader_collate_fn else batch

    loader = DataLoader(microbatch_ids, batch_size=dataloader_batch_size, sampler=sampler,
                        num_workers=dataloader_num_workers, collate_fn=collate, pin_memory=dataloader_pin_memory)
    io_kwargs = dict(dataset=microbatch_ids, batch_size=dataloader_batch_size, pin_memory=dataloader_pin_memory,
                     data_sampler=sampler, collate_fn=collate, num_local_io_workers=dataloader_num_workers)
    return loader, io_kwargs


class VariableBatchSizeLR(torch.optim.lr_scheduler.LRScheduler):
    """Wraps an LR scheduler; after each step the LR of every group is the wrapped LR scaled to the size of the
    batch that is about to run."""

    def __init__(self, lr_scheduler, base_batch_size, batch_sizes, dataloader, lr_scaling_method="linear",
                 last_epoch=-1, verbose=False):
        self.base_lr_scheduler = lr_scheduler
        self.base_batch_size = base_batch_size
        self.batch_sizes = list(batch_sizes)
        self.dataloader = dataloader
        self.lr_scaling_method = lr_scaling_method
        self.base_lrs = list(lr_scheduler.get_last_lr() if hasattr(lr_scheduler, "get_last_lr") else
                             lr_scheduler.get_lr())
        self.last_epoch = last_epoch
        self.verbose = verbose
        self._last_lr = list(self.base_lrs)
        self.step(0)

    @property
    def optimizer(self):
        return self.base_lr_scheduler.optimizer

    def state_dict(self):
        return {"base_lr_scheduler": self.base_lr_scheduler.state_dict(), "base_batch_size": self.base_batch_size,
                "lr_scaling_method": self.lr_scaling_method, "batch_sizes": self.batch_sizes,
                "base_lrs": self.base_lrs, "last_epoch": self.last_epoch}

    def load_state_dict(self, sd):
        self.base_lr_scheduler.load_state_dict(sd["base_lr_scheduler"])
        for k in ("base_batch_size", "lr_scaling_method", "batch_sizes", "base_lrs", "last_epoch"):
            setattr(self, k, sd[k])

    def get_last_lr(self):
        return self._last_lr

    def get_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def step(self, epoch=None):
        # the wrapped scheduler advances after the first call (which only scales the initial LR)
        if epoch is None or epoch > 0:
            self.base_lr_scheduler.step()
        self.last_epoch = self.last_epoch + 1 if epoch is None else epoch
        bs = self.batch_sizes[min(max(self.last_epoch, 0), len(self.batch_sizes) - 1)]
        base = (self.base_lr_scheduler.get_last_lr() if hasattr(self.base_lr_scheduler, "get_last_lr") else
                self.base_lr_scheduler.get_lr())
        self._last_lr = []
        for g, lr in zip(self.optimizer.param_groups, base):
            g["lr"] = scale_lr(self.base_batch_size, bs, lr, self.lr_scaling_method)
            self._last_lr.append(g["lr"])


def lr_scheduler_for_variable_batch_size(base_batch_size, batch_sizes, dataloader, lr_scheduler_or_optimizer,
                                         lr_scaling_method="linear"):
    """Accepts an LR scheduler, or an optimizer (then a constant base schedule is assumed)."""
    sched = lr_scheduler_or_optimizer
    if isinstance(sched, torch.optim.Optimizer):
        sched = torch.optim.lr_scheduler.LambdaLR(sched, lambda _: 1.0)
    return VariableBatchSizeLR(sched, base_batch_size, batch_sizes, dataloader, lr_scaling_method)


def get_dataloader_and_lr_scheduler_for_variable_batch_size(dataset, dataset_seqlens, max_tokens,
                                                            effective_batch_size, dataset_filter_ids=None,
                                                            lr_scaling_method="linear", min_batch_size=1,
                                                            max_batch_size=None, sequence_picking_order="dataloader",
                                                            dataloader_batch_size=1, dataloader_rank=0,
                                                            dataloader_num_replicas=1, dataloader_num_workers=0,
                                                            dataloader_collate_fn=None, dataloader_pin_memory=False,
                                                            optimizer=None, lr_scheduler_class=None,
                                                            lr_scheduler_kwargs=None,
                                                            required_microbatches_of_same_size=False,
                                                            required_microbatches_of_same_seqlen=False,
                                                            sample_padding_fn=None, verbose=False, seed=None):
    mb_ids, batch_sizes, batch_max_seqlens = batch_by_seqlens(
        dataset_seqlens, max_tokens, sequence_ids_per_mb=dataset_filter_ids, min_batch_size=min_batch_size,
        max_batch_size=max_batch_size, sequence_picking_order=sequence_picking_order,
        effective_batch_size=effective_batch_size,
        required_microbatches_of_same_size=required_microbatches_of_same_size, verbose=verbose, seed=seed)
    loader, _ = dataloader_for_variable_batch_size(
        dataset, mb_ids, batch_max_seqlens, dataloader_rank=dataloader_rank,
        dataloader_batch_size=dataloader_batch_size, dataloader_num_replicas=dataloader_num_replicas,
        dataloader_collate_fn=dataloader_collate_fn, dataloader_num_workers=dataloader_num_workers,
        dataloader_pin_memory=dataloader_pin_memory,
        required_microbatches_of_same_seqlen=required_microbatches_of_same_seqlen,
        sample_padding_fn=sample_padding_fn)
    sched = None
    if optimizer is not None:
        base = (lr_scheduler_class(optimizer, **(lr_scheduler_kwargs or {})) if lr_scheduler_class is not None
                else optimizer)
        sched = lr_scheduler_for_variable_batch_size(max_tokens, batch_sizes, loader, base, lr_scaling_method)
    return loader, sched


def get_dataloader_and_lr_scheduler_for_variable_batch_size_deepspeed(dataset, engine, dataset_seqlens=None,
                                                                      dataset_filter_ids=None, dataloader_rank=None,
                                                                      dataloader_num_replicas=None, **kwargs):
    """Engine-aware variant: the engine's data-efficiency config supplies the token budget and the DP layout."""
    cfg = getattr(engine, "config", None)
    de = getattr(cfg, "data_efficiency", None) or {}
    vb = de.get("data_sampling", {}).get("dynamic_batching", {}) if isinstance(de, dict) else {}
    max_tokens = kwargs.pop("max_tokens", vb.get("max_tokens", 2048))
    dp = engine.dp_world_size if hasattr(engine, "dp_world_size") else 1
    rank = engine.global_rank if hasattr(engine, "global_rank") else 0
    gas = engine.gradient_accumulation_steps() if hasattr(engine, "gradient_accumulation_steps") else 1
    if dataset_seqlens is None:
        dataset_seqlens = [len(dataset[i]) for i in range(len(dataset))]
    return get_dataloader_and_lr_scheduler_for_variable_batch_size(
        dataset, dataset_seqlens, max_tokens, effective_batch_size=dp * gas, dataset_filter_ids=dataset_filter_ids,
        lr_scaling_method=vb.get("lr_scaling_method", kwargs.pop("lr_scaling_method", "linear")),
        min_batch_size=vb.get("min_batch_size", 1), max_batch_size=vb.get("max_batch_size"),
        sequence_picking_order=vb.get("sequence_picking_order", "dataloader"),
        dataloader_rank=rank if dataloader_rank is None else dataloader_rank,
        dataloader_num_replicas=dp if dataloader_num_replicas is None else dataloader_num_replicas,
        optimizer=getattr(engine, "optimizer", None), **kwargs)
