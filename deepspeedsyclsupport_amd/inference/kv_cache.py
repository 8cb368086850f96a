"""Blocked (paged) KV cache shared by the v1 kernel-injected engine and the v2 ragged engine
(reference `inference/v2/ragged/{kv_cache.py:40, blocked_allocator.py:11}` and the v1 in-workspace cache of
`csrc/transformer/inference/csrc/pt_binding.cpp:434-557`).

Per layer the cache is two tensors [num_blocks, kv_heads, block_size, head_dim] (head-major inside a block, so the
decode kernel reads one head's keys contiguously). Sequences own lists of block ids; the allocator is a simple
host-side free list (block ids are plain ints, the per-sequence block table is mirrored to a device int32 tensor).
Sized from free HBM: with 288 GB per MI355X even a 70B model leaves >100 GB of cache.
"""
import torch


class BlockedAllocator:

    def __init__(self, num_blocks):
        self.num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))

    @property
    def free_blocks(self):
        return len(self._free)

    def allocate(self, n):
        if n > len(self._free):
            raise ValueError(f"KV cache exhausted: need {n} blocks, {len(self._free)} free")
        out = [self._free.pop() for _ in range(n)]
        return out

    def free(self, blocks):
        for b in blocks:
            self._free.append(int(b))


class BlockedKVCache:

    def __init__(self, num_layers, num_blocks, kv_heads, block_size, head_dim, dtype, device):
        self.num_layers = num_layers
        self.num_blocks = num_blocks
        self.kv_heads = kv_heads
        self.block_size = block_size
        self.head_dim = head_dim
        self.dtype = dtype
        self.device = device
        shape = (num_blocks, kv_heads, block_size, head_dim)
        self.k = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(num_layers)]
        self.v = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(num_layers)]
        self.allocator = BlockedAllocator(num_blocks)

    @staticmethod
    def blocks_for_memory(bytes_avail, num_layers, kv_heads, block_size, head_dim, dtype):
        per_block = 2 * num_layers * kv_heads * block_size * head_dim * torch.tensor([], dtype=dtype).element_size()
        return max(int(bytes_avail // per_block), 1)

    def bytes(self):
        return 2 * sum(t.numel() * t.element_size() for t in self.k)

    # ---- the reference's cache-object interface (`inference/v2/ragged/kv_cache.py:40-208`)
    @property
    def num_caches(self):
        """Cache groups (models with several attention geometries would hold one each): one here."""
        return 1

    @property
    def free_blocks(self):
        return torch.tensor([self.allocator.free_blocks], dtype=torch.int32)

    def reserve(self, num_blocks, cache_group=0):
        """Take `num_blocks` block ids out of the free list."""
        return torch.tensor(self.allocator.allocate(int(num_blocks)), dtype=torch.int32)

    def free(self, blocks, cache_group=0):
        self.allocator.free(blocks.tolist() if torch.is_tensor(blocks) else blocks)

    def get_cache(self, cache_id, cache_group=0):
        """(keys, values) of layer `cache_id`, each [blocks, kv_heads, block_size, head_dim]."""
        return self.k[cache_id], self.v[cache_id]

    def offload(self, blocks, cache_group=0):
        """Copy the given blocks of every layer to pinned host memory (the blocks stay allocated); returns the
        handle `restore` takes."""
        idx = torch.as_tensor(blocks, dtype=torch.long, device=self.k[0].device)
        pin = torch.device(self.device).type == "cuda" if self.device is not None else False
        host = []
        for k, v in zip(self.k, self.v):
            hk = torch.empty((idx.numel(), ) + tuple(k.shape[1:]), dtype=k.dtype, pin_memory=pin)
            hv = torch.empty_like(hk, pin_memory=pin)
            hk.copy_(k.index_select(0, idx), non_blocking=pin)
            hv.copy_(v.index_select(0, idx), non_blocking=pin)
            host.append((hk, hv))
        if pin:
            torch.cuda.current_stream().synchronize()
        return {"blocks": idx.cpu(), "data": host}

    def restore(self, handle, blocks=None, cache_group=0):
        """Write offloaded blocks back, to their old ids or to `blocks` (same count)."""
        idx = torch.as_tensor(handle["blocks"] if blocks is None else blocks, dtype=torch.long,
                              device=self.k[0].device)
        for (hk, hv), k, v in zip(handle["data"], self.k, self.v):
            k.index_copy_(0, idx, hk.to(k.device, non_blocking=True))
            v.index_copy_(0, idx, hv.to(v.device, non_blocking=True))


def split_kv(kv_cache):
    """(keys, values) of a stacked [2, ...] cache tensor or an already split pair."""
    return kv_cache[0], kv_cache[1]


class SequenceState:
    """Per-sequence bookkeeping: tokens already in cache and owned block ids."""

    def __init__(self, uid, block_size):
        self.uid = uid
        self.seen_tokens = 0
        self.blocks = []
        self.block_size = block_size

    def blocks_needed(self, new_tokens):
        total = self.seen_tokens + new_tokens
        need = (total + self.block_size - 1) // self.block_size
        return max(0, need - len(self.blocks))
