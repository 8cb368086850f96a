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
    """Reference `runtime/dataloader.py:41-160`. Three modes: curriculum learning (`deepspeed_dataloader_config`
    built by the engine from `data_efficiency.data_sampling`: a `DeepSpeedDataSampler` hands out difficulty-filtered
    micro-batches as a batch sampler), one process per device (`local_rank >= 0`: DistributedSampler over the
    data-parallel ranks), or one process driving every visible device (`local_rank < 0`: the batch is scaled by
    the device count). Host loader workers default to 2 per device."""

    def __init__(self, dataset, batch_size, pin_memory, local_rank, tput_timer, collate_fn=None,
                 num_local_io_workers=None, data_sampler=None, data_parallel_world_size=None,
                 data_parallel_rank=None, dataloader_drop_last=False, deepspeed_dataloader_config={}):
        from ..accelerator import get_accelerator
        self.deepspeed_dataloader_config = deepspeed_dataloader_config or {}
        self.tput_timer = tput_timer
        self.curriculum_learning_enabled = bool(self.deepspeed_dataloader_config.get("curriculum_learning", False))
        if self.curriculum_learning_enabled:
            from .data_pipeline.data_sampling.data_sampler import DeepSpeedDataSampler
            c = self.deepspeed_dataloader_config
            data_sampler = DeepSpeedDataSampler(c["data_efficiency"], len(dataset), batch_size, data_parallel_rank,
                                                data_parallel_world_size,
                                                gradient_accumulation_steps=c.get("gradient_accumulation_steps", 1),
                                                global_rank=c.get("global_rank", 0),
                                                drop_last=dataloader_drop_last)
            device_count = 1
            num_local_io_workers = c.get("data_sampling_num_workers", 0)
        else:
            if local_rank is not None and local_rank >= 0:
                if data_sampler is None:
                    if data_parallel_world_size and data_parallel_world_size > 1:
                        data_sampler = DistributedSampler(dataset, num_replicas=data_parallel_world_size,
                                                          rank=data_parallel_rank)
                    else:
                        data_sampler = RandomSampler(dataset)
                device_count = 1
            else:
                if data_sampler is None:
                    data_sampler = RandomSampler(dataset)
                device_count = max(get_accelerator().device_count(), 1)
                batch_size *= device_count
            if num_local_io_workers is None:
                num_local_io_workers = 2 * device_count
        self.batch_size = batch_size
        self.device_count = device_count
        self.data_sampler = data_sampler
        self.dataset = dataset
        self.collate_fn = collate_fn
        self.num_local_io_workers = int(num_local_io_workers)
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
        data = next(self.data)
        if self.curriculum_learning_enabled and self.post_process_func is not None:
            data = self.post_process_func(data, self.data_sampler.state_dict())
        return data

    def _create_dataloader(self):
        kw = dict(pin_memory=self.pin_memory, num_workers=self.num_local_io_workers)
        if self.curriculum_learning_enabled:
            kw["batch_sampler"] = self.data_sampler
        else:
            kw.update(batch_size=self.batch_size, sampler=self.data_sampler, drop_last=self.drop_last)
        if self.collate_fn is not None:
            kw["collate_fn"] = self.collate_fn
        self.dataloader = DataLoader(self.dataset, **kw)
        self.data = iter(self.dataloader)
        return self.dataloader
