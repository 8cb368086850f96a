"""Per-sequence KV bookkeeping of the ragged engine (reference `inference/v2/ragged/sequence_descriptor.py`)."""


class BaseSequenceDescriptor:
    """What the scheduler needs to know about a sequence: tokens already in the KV cache and blocks it owns."""

    @property
    def seen_tokens(self) -> int:
        raise NotImplementedError()

    @property
    def cur_allocated_blocks(self) -> int:
        raise NotImplementedError()

    def kv_blocks_ptr(self, cache_group=0):
        raise NotImplementedError()


class DSSequenceDescriptor(BaseSequenceDescriptor):

    def __init__(self, uid, block_size):
        self.uid = uid
        self._seen_tokens = 0
        self.in_flight_tokens = 0
        self.blocks = []
        self.block_size = block_size

    @property
    def tracking_id(self):
        return self.uid

    @property
    def seen_tokens(self):
        return self._seen_tokens

    @seen_tokens.setter
    def seen_tokens(self, n):
        self._seen_tokens = n

    @property
    def cur_allocated_blocks(self):
        return len(self.blocks)

    @property
    def max_context(self):
        """Tokens the blocks owned so far can hold."""
        return len(self.blocks) * self.block_size

    @property
    def all_block_ids(self):
        return list(self.blocks)

    def free_kv_cache(self, free_ids, cache_group=0):
        """Forget blocks handed back to the allocator (sliding-window models release the oldest ones)."""
        drop = {int(i) for i in free_ids}
        self.blocks = [b for b in self.blocks if b not in drop]

    def kv_cache_ids(self, cache_group=0, on_device=False):
        return self.blocks

    def kv_blocks_ptr(self, cache_group=0):
        return self.blocks

    def extend_kv_cache(self, new_ids, cache_group=0):
        self.blocks.extend(int(i) for i in new_ids)

    def blocks_needed(self, new_tokens):
        total = self._seen_tokens + new_tokens
        return max(0, -(-total // self.block_size) - len(self.blocks))

    def pre_forward(self, n):
        self.in_flight_tokens = n

    def post_forward(self):
        self._seen_tokens += self.in_flight_tokens
        self.in_flight_tokens = 0


class PlaceholderSequenceDescriptor(DSSequenceDescriptor):
    """Stands in for a sequence the engine does not track yet (scheduling queries about new sequences)."""

    def __init__(self, block_size=64):
        super().__init__(-1, block_size)
