"""Sequence tracking and KV-block allocation (reference `inference/v2/ragged/ragged_manager.py:19`)."""
import torch

from ...kv_cache import BlockedAllocator
from .sequence_descriptor import DSSequenceDescriptor


class DSStateManager:

    def __init__(self, config, num_blocks, block_size):
        self.config = config
        self.block_size = block_size
        self.allocator = BlockedAllocator(num_blocks)
        self._seqs = {}
        self._kv_cache = None

    @property
    def n_tracked_sequences(self):
        return len(self._seqs)

    @property
    def tracked_sequences(self):
        return self._seqs

    @property
    def free_blocks(self):
        return self.allocator.free_blocks

    @property
    def kv_block_size(self):
        return self.block_size

    @property
    def n_kv_cache_groups(self):
        return 1

    def attach_cache(self, kv_cache):
        """The model's `BlockedKVCache` (set by the engine once the model has allocated it)."""
        self._kv_cache = kv_cache
        if kv_cache is not None and getattr(kv_cache, "allocator", None) is not None \
                and kv_cache.allocator.num_blocks == self.allocator.num_blocks:
            self.allocator = kv_cache.allocator   # one free list for `cache.reserve / free` and the manager

    def get_cache(self, cache_id, cache_group=0):
        """(keys, values) of layer `cache_id`."""
        return self._kv_cache.get_cache(cache_id, cache_group)

    def query(self, uid=None):
        """The tracked sequence `uid`, or None."""
        return self._seqs.get(uid)

    def get_sequence(self, uid):
        return self._seqs.get(uid)

    def get_or_create_sequence(self, uid):
        seq = self._seqs.get(uid)
        if seq is None:
            if len(self._seqs) >= self.config.max_tracked_sequences:
                raise RuntimeError("engine is tracking max_tracked_sequences sequences")
            seq = self._seqs[uid] = DSSequenceDescriptor(uid, self.block_size)
        return seq

    def allocate_blocks(self, seq, n_tokens):
        need = seq.blocks_needed(n_tokens)
        if need:
            seq.extend_kv_cache(self.allocator.allocate(need))

    def flush_sequence(self, uid):
        seq = self._seqs.pop(uid, None)
        if seq is not None:
            self.allocator.free(seq.blocks)
            seq.blocks = []

    def block_table(self, seqs, device):
        width = max(len(s.blocks) for s in seqs)
        bt = torch.zeros(len(seqs), width, dtype=torch.int32)
        for i, s in enumerate(seqs):
            bt[i, :len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
        return bt.to(device)
