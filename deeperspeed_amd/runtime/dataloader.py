"""Engine-owned data loading.

Behaviour of reference deepspeed/runtime/dataloader.py:10-99: `RepeatingLoader` restarts
an exhausted iterator; `DeepSpeedDataLoader` shards the dataset over the data-parallel
ranks with a `DistributedSampler` (one process per GPU, local_rank >= 0) or samples
randomly with the batch widened to every visible device (single-process mode), defaults to
two loader workers per device, and starts the engine's throughput timer on every batch.

MI355X notes: batches are produced on pinned host memory (`pin_memory`) so the engine's
H2D copy is asynchronous; the torch DataLoader is built lazily on each `iter()`.
"""

import torch
from torch.utils.data import DataLoader, RandomSampler
from torch.utils.data.distributed import DistributedSampler


class RepeatingLoader:
    """Endless iterator over `loader`: a StopIteration re-creates the underlying iterator."""

    def __init__(self, loader):
        self.loader = loader
        self.data_iter = iter(loader)

    def __iter__(self):
        return self

    def __next__(self):
        for attempt in range(2):
            try:
                return next(self.data_iter)
            except StopIteration:
                if attempt:
                    raise
                self.data_iter = iter(self.loader)


def _default_sampler(dataset, per_process, world, rank):
    if per_process:
        return DistributedSampler(dataset=dataset, num_replicas=world, rank=rank)
    return RandomSampler(dataset)


class DeepSpeedDataLoader:
    def __init__(self, dataset, batch_size, pin_memory, local_rank, tput_timer, collate_fn=None,
                 num_local_io_workers=None, data_sampler=None, data_parallel_world_size=None,
                 data_parallel_rank=None):
        per_process = local_rank >= 0  # launched one process per GPU
        self.device_count = 1 if per_process else max(1, torch.cuda.device_count())
        self.batch_size = batch_size * self.device_count
        self.data_sampler = data_sampler if data_sampler is not None else \
            _default_sampler(dataset, per_process, data_parallel_world_size, data_parallel_rank)
        self.num_local_io_workers = 2 * self.device_count if num_local_io_workers is None else num_local_io_workers
        self.dataset = dataset
        self.collate_fn = collate_fn
        self.pin_memory = pin_memory
        self.tput_timer = tput_timer
        self.len = len(self.data_sampler)
        self.dataloader = None
        self.data = None

    def __len__(self):
        return self.len

    def __iter__(self):
        self._create_dataloader()
        return self

    def __next__(self):
        if self.tput_timer is not None:
            self.tput_timer.start()
        return next(self.data)

    def _create_dataloader(self):
        extra = {} if self.collate_fn is None else {"collate_fn": self.collate_fn}
        self.dataloader = DataLoader(self.dataset, batch_size=self.batch_size, sampler=self.data_sampler,
                                     pin_memory=self.pin_memory, num_workers=self.num_local_io_workers, **extra)
        self.data = iter(self.dataloader)
        return self.dataloader
