"""NVMe home for offloaded ZeRO-3 parameter partitions (reference `runtime/swap_tensor/partitioned_param_swapper.py:36`
`AsyncPartitionedParameterSwapper`, config `offload_param.device = "nvme"`).

Each flat group's bf16 shard is one file `<nvme_path>/zero_stage_3/params/rank<r>/group<i>.param.swp`, mapped into
the address space with MAP_SHARED (`torch.from_file(shared=True)`). The optimizer writes the updated shard through
the mapping after every step and the fetch path copies it to the device on the all-gather stream; the kernel's page
cache provides read-ahead and write-back, so host RAM only holds the pages in flight instead of 2 bytes per
parameter, and nothing has to be pinned. (The optimizer-state side uses the explicit double-buffered aio pipeline of
`optimizer_swapper.py`, where chunk-wise streaming through a CPU Adam needs it.)
"""
import os

import torch


class ParamNvmeStore:

    def __init__(self, folder):
        os.makedirs(folder, exist_ok=True)
        self.folder = folder
        self.paths = {}

    def path(self, idx):
        return os.path.join(self.folder, f"group{idx}.param.swp")

    def create(self, idx, init):
        """Create (or overwrite) the file for group `idx` and return a file-backed host tensor holding `init`."""
        path = self.path(idx)
        n = init.numel()
        nbytes = n * init.element_size()
        with open(path, "wb") as f:
            f.truncate(nbytes)
        t = torch.from_file(path, shared=True, size=n, dtype=init.dtype)
        t.copy_(init.reshape(-1))
        self.paths[idx] = path
        return t

    def bytes_on_disk(self):
        return sum(os.path.getsize(p) for p in self.paths.values() if os.path.exists(p))
