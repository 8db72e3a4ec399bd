"""Data loading helpers (reference: runtime/dataloader.py -- DeepSpeedDataLoader :41, RepeatingLoader :17)."""
import torch
from torch.utils.data import DataLoader, DistributedSampler


class RepeatingLoader:

    def __init__(self, loader):
        self.loader = loader
        self.data_iter = iter(self.loader)

    def __iter__(self):
        return self

    def __next__(self):
        try:
            return next(self.data_iter)
        except StopIteration:
            self.data_iter = iter(self.loader)
            return next(self.data_iter)


class DeepSpeedDataLoader:
    """DataLoader over the DP rank's slice of the dataset (DistributedSampler), pinned memory on GPU."""

    def __init__(self, dataset, batch_size, pin_memory=None, local_rank=0, tput_timer=None, collate_fn=None,
                 num_local_io_workers=None, data_sampler=None, data_parallel_world_size=1, data_parallel_rank=0,
                 dataloader_drop_last=False, deepspeed_dataloader_config=None):
        if data_sampler is None and data_parallel_world_size > 1:
            data_sampler = DistributedSampler(dataset, num_replicas=data_parallel_world_size, rank=data_parallel_rank)
        self.sampler = data_sampler
        self.tput_timer = tput_timer
        self.batch_size = batch_size
        if pin_memory is None:
            pin_memory = torch.cuda.is_available()
        self.dataloader = DataLoader(dataset, batch_size=batch_size, sampler=data_sampler, collate_fn=collate_fn,
                                     pin_memory=pin_memory, num_workers=num_local_io_workers or 0,
                                     drop_last=dataloader_drop_last, shuffle=False if data_sampler else False)
        self.len = len(self.dataloader)
        self.data = None

    def __iter__(self):
        self.data = iter(self.dataloader)
        return self

    def __len__(self):
        return self.len

    def __next__(self):
        if self.tput_timer:
            self.tput_timer.start()
        return next(self.data)
