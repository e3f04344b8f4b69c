"""Data loading (parity: reference runtime/dataloader.py:17 RepeatingLoader, :41 DeepSpeedDataLoader).

Samples are sharded over the *data-parallel* ranks only: ranks of one sequence- or tensor-parallel
group read the same batch."""
import torch
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler


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
            if hasattr(self.loader, "sampler") and hasattr(self.loader.sampler, "set_epoch"):
                self.loader.sampler.set_epoch(getattr(self.loader.sampler, "epoch", 0) + 1)
            self.data_iter = iter(self.loader)
            return next(self.data_iter)


class SXEDataLoader:
    def __init__(self, dataset, batch_size, pin_memory=False, collate_fn=None, num_workers=0,
                 data_parallel_world_size=1, data_parallel_rank=0, data_sampler=None, drop_last=False,
                 shuffle=True, seed=0):
        self.dataset = dataset
        if data_sampler is None:
            data_sampler = DistributedSampler(dataset, num_replicas=data_parallel_world_size, rank=data_parallel_rank,
                                              shuffle=shuffle, seed=seed, drop_last=drop_last)
        self.data_sampler = data_sampler
        self.batch_size = batch_size
        self.dataloader = DataLoader(dataset, batch_size=batch_size, sampler=data_sampler, collate_fn=collate_fn,
                                     pin_memory=pin_memory, num_workers=num_workers, drop_last=drop_last)
        self.len = len(self.dataloader)
        self.epoch = 0
        # engine.set_data_post_process_func (reference runtime/dataloader.py:100,120): called on every
        # batch with the sampler's state (the curriculum difficulty) before the batch is returned
        self.post_process_func = None

    def __len__(self):
        return self.len

    def __iter__(self):
        if hasattr(self.data_sampler, "set_epoch"):
            self.data_sampler.set_epoch(self.epoch)
        self.epoch += 1
        it = iter(self.dataloader)
        if self.post_process_func is None:
            return it
        return self._post_processed(it)

    def _post_processed(self, it):
        for batch in it:
            state = self.data_sampler.state_dict() if hasattr(self.data_sampler, "state_dict") else {}
            yield self.post_process_func(batch, state)


DeepSpeedDataLoader = SXEDataLoader
