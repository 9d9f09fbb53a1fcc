"""Engine-owned data loading (reference parity: deepspeed/runtime/dataloader.py:10-99)."""

import torch
from torch.utils.data import DataLoader, RandomSampler
from torch.utils.data.distributed import DistributedSampler


class RepeatingLoader:
    """Wraps an iterator to restart it transparently at the end (for step-based training)."""

    def __init__(self, loader):
        self.loader = loader
        self.data_iter = iter(self.loader)

    def __iter__(self):
        return self

    def __next__(self):
        try:
            batch = next(self.data_iter)
        except StopIteration:
            self.data_iter = iter(self.loader)
            batch = next(self.data_iter)
        return batch


class DeepSpeedDataLoader:
    def __init__(self, dataset, batch_size, pin_memory, local_rank, tput_timer, collate_fn=None, num_local_io_workers=None,
                 data_sampler=None, data_parallel_world_size=None, data_parallel_rank=None):
        self.tput_timer = tput_timer
        self.batch_size = batch_size
        if local_rank >= 0:
            if data_sampler is None:
                data_sampler = DistributedSampler(dataset=dataset, num_replicas=data_parallel_world_size,
                                                  rank=data_parallel_rank)
            device_count = 1
        else:
            if data_sampler is None:
                data_sampler = RandomSampler(dataset)
            device_count = max(1, torch.cuda.device_count())
            batch_size *= device_count
        if num_local_io_workers is None:
            num_local_io_workers = 2 * device_count
        self.num_local_io_workers = num_local_io_workers
        self.data_sampler = data_sampler
        self.dataset = dataset
        self.collate_fn = collate_fn
        self.device_count = device_count
        self.pin_memory = pin_memory
        self.len = len(self.data_sampler)
        self.data = None

    def __iter__(self):
        self._create_dataloader()
        return self

    def __len__(self):
        return self.len

    def __next__(self):
        if self.tput_timer:
            self.tput_timer.start()
        return next(self.data)

    def _create_dataloader(self):
        kw = dict(batch_size=self.batch_size, pin_memory=self.pin_memory, sampler=self.data_sampler,
                  num_workers=self.num_local_io_workers)
        if self.collate_fn is not None:
            kw["collate_fn"] = self.collate_fn
        self.dataloader = DataLoader(self.dataset, **kw)
        self.data = (x for x in self.dataloader)
        return self.dataloader
