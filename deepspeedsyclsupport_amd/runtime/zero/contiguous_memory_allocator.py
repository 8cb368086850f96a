"""Defragmenting sub-allocator over one preallocated buffer (reference
`runtime/zero/contiguous_memory_allocator.py`).

Tensors are handed out as views of a single flat buffer. When the free space is large enough in total but not in one
piece, live tensors are slid towards the start of the buffer (their registered parameters' `.data` re-pointed) until
a hole of the requested size opens. Used for activation-checkpoint buffers and gathered-parameter staging, where
sizes repeat every step and `hipMalloc` / caching-allocator fragmentation would otherwise creep.
"""
import torch


class ContiguousMemoryAllocator:

    def __init__(self, size, dtype, device):
        self.buffer = torch.zeros(size, dtype=dtype, device=device)
        self.size = size
        self.total_free = size
        self.largest_contiguous = size
        self.max_allocated = 0
        self._free = {0: size}          # start -> length
        self._live = {}                 # tensor id -> (start, length, tensor)
        self._param_of = {}             # tensor id -> parameter whose .data is this tensor

    # ------------------------------------------------------------------------------------------ public
    def allocate_tensor(self, size):
        if size > self.total_free:
            raise MemoryError(f"Not enough memory in buffer. Allocation failed: asked {size}, free "
                              f"{self.total_free}")
        if size > self.largest_contiguous:
            self._defragment(size)
        start = self._first_fit(size)
        length = self._free.pop(start)
        if length > size:
            self._free[start + size] = length - size
        t = self.buffer.narrow(0, start, size)
        self._live[id(t)] = (start, size, t)
        self.total_free -= size
        self.max_allocated = max(self.max_allocated, self.size - self.total_free)
        self._refresh()
        return t

    def assign_to_param(self, tensor, param, numel, shape):
        """Make `param.data` a view of `tensor` (allocated here); defragmentation keeps it pointing at the data."""
        if id(tensor) not in self._live:
            raise ValueError("No such tensor allocated by the allocator.")
        self._param_of[id(tensor)] = (param, numel, tuple(shape))
        param.data = tensor.narrow(0, 0, numel).view(shape)

    def release_tensor(self, tensor):
        key = id(tensor)
        if key not in self._live:
            raise ValueError("No such tensor allocated by the allocator.")
        start, size, _ = self._live.pop(key)
        self._param_of.pop(key, None)
        self._free[start] = size
        self.total_free += size
        self._merge()
        self._refresh()

    def release_tensor_with_id(self, tensor_id):
        for key, (_, _, t) in list(self._live.items()):
            if key == tensor_id:
                return self.release_tensor(t)
        raise ValueError("No such tensor allocated by the allocator.")

    def print_allocation(self, resolution=200):
        cells = ["."] * resolution
        for start, size, _ in self._live.values():
            for c in range(start * resolution // self.size, max(start * resolution // self.size + 1,
                                                                (start + size) * resolution // self.size)):
                cells[min(c, resolution - 1)] = "x"
        print("".join(cells))

    def max_allocated_size(self):
        return self.max_allocated

    # ------------------------------------------------------------------------------------------ internals
    def _first_fit(self, size):
        for start in sorted(self._free):
            if self._free[start] >= size:
                return start
        raise MemoryError("no contiguous block after defragmentation")

    def _merge(self):
        merged, prev = {}, None
        for start in sorted(self._free):
            if prev is not None and prev + merged[prev] == start:
                merged[prev] += self._free[start]
            else:
                merged[start] = self._free[start]
                prev = start
        self._free = merged

    def _refresh(self):
        self.largest_contiguous = max(self._free.values(), default=0)

    def _defragment(self, need):
        """Slide live tensors down, lowest first, until a free block of `need` elements exists."""
        cursor = 0
        for key in sorted(self._live, key=lambda k: self._live[k][0]):
            start, size, t = self._live[key]
            if start != cursor:
                dst = self.buffer.narrow(0, cursor, size)
                if cursor + size <= start:
                    dst.copy_(t)
                else:                      # overlapping move: go through a temporary
                    dst.copy_(t.clone())
                t.set_(self.buffer.untyped_storage(), self.buffer.storage_offset() + cursor, (size, ), (1, ))
                self._live[key] = (cursor, size, t)
                if key in self._param_of:
                    param, numel, shape = self._param_of[key]
                    param.data = t.narrow(0, 0, numel).view(shape)
            cursor += size
        self._free = {cursor: self.size - cursor} if cursor < self.size else {}
        self._refresh()
        if self.largest_contiguous < need:
            raise MemoryError("defragmentation could not open a large enough block")
