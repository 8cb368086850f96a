"""DeepSpeedDataLoader / RepeatingLoader (reference `runtime/dataloader.py:17-162`): DistributedSampler over the
data-parallel rank, pinned host batches so the H2D copy can overlap (non_blocking)."""
import torch
from torch.utils.data import DataLoader, RandomSampler
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
            self.data_iter = iter(self.loader)
            return next(self.data_iter)


class DeepSpeedDataLoader:

    def __init__(self, dataset, batch_size, pin_memory, local_rank, tput_timer, collate_fn=None,
                 num_local_io_workers=None, data_sampler=None, data_parallel_world_size=None,
                 data_parallel_rank=None, dataloader_drop_last=False, deepspeed_dataloader_config={}):
        self.tput_timer = tput_timer
        self.batch_size = batch_size
        if data_sampler is None:
            if data_parallel_world_size and data_parallel_world_size > 1:
                data_sampler = DistributedSampler(dataset, num_replicas=data_parallel_world_size,
                                                  rank=data_parallel_rank)
            else:
                data_sampler = RandomSampler(dataset)
        self.data_sampler = data_sampler
        self.dataset = dataset
        self.collate_fn = collate_fn
        self.num_local_io_workers = num_local_io_workers or 0
        self.pin_memory = pin_memory
        self.drop_last = dataloader_drop_last
        self.len = len(self.data_sampler) // batch_size if self.drop_last else \
            (len(self.data_sampler) + batch_size - 1) // batch_size
        self.dataloader = None
        self.data = None
        self.post_process_func = None

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
                  num_workers=self.num_local_io_workers, drop_last=self.drop_last)
        if self.collate_fn is not None:
            kw["collate_fn"] = self.collate_fn
        self.dataloader = DataLoader(self.dataset, **kw)
        self.data = (x for x in self.dataloader)
        return self.dataloader
