"""Helpers of the NVMe swappers (reference `runtime/swap_tensor/utils.py`): aligned sizes, per-tensor swap
bookkeeping and a pool of equal-sized slices of one pinned buffer."""
import torch

from ...utils.logging import logger

MIN_AIO_BYTES = 1024**2
AIO_ALIGNED_BYTES = 1024


def swap_in_tensors(swap_handle, tensor_buffers, swap_paths):
    for buffer, path in zip(tensor_buffers, swap_paths):
        assert swap_handle.async_pread(buffer, path) == 0


def swap_out_tensors(swap_handle, tensor_buffers, swap_paths):
    for buffer, path in zip(tensor_buffers, swap_paths):
        assert swap_handle.async_pwrite(buffer, path) == 0


def print_object(obj, name, exclude_list=()):
    logger.info("{}:".format(name))
    for arg in sorted(vars(obj)):
        if arg not in exclude_list:
            logger.info("  {} {} {}".format(arg, "." * (29 - len(arg)), getattr(obj, arg)))


def get_sized_buffer(buffer, num_elems):
    assert num_elems <= buffer.numel(), f"num_elems {num_elems} > buffer {buffer.numel()}"
    return buffer.narrow(0, 0, num_elems) if num_elems < buffer.numel() else buffer


def get_sized_buffers(buffer_list, num_elems_list):
    return [get_sized_buffer(b, n) for b, n in zip(buffer_list, num_elems_list)]


class SwapBuffer:
    """One slice of the pool: tensors are packed into it back to back, each padded to the I/O alignment."""

    def __init__(self, buffer):
        self.buffer = buffer
        self.reset()

    def reset(self):
        self.offset = 0
        self.swap_tensors, self.compute_tensors, self.swap_paths = {}, {}, {}
        self.num_elem = 0

    def insert_tensor(self, tensor, swap_path, aligned_numel):
        swap_tensor, compute_tensor = self.allocate_tensor(swap_path, tensor.numel(), aligned_numel)
        compute_tensor.data.copy_(tensor.data)
        return swap_tensor, compute_tensor

    def allocate_tensor(self, swap_path, numel, aligned_numel):
        assert self.has_space(aligned_numel)
        assert self.offset not in self.swap_tensors
        swap_tensor = self.buffer.narrow(0, self.offset, aligned_numel)
        compute_tensor = swap_tensor.narrow(0, 0, numel)
        self.swap_tensors[self.offset], self.compute_tensors[self.offset] = swap_tensor, compute_tensor
        self.swap_paths[self.offset] = swap_path
        self.offset += aligned_numel
        self.num_elem += numel
        return swap_tensor, compute_tensor

    def has_space(self, numel):
        return self.offset + numel <= self.buffer.numel()

    def get_swap_tensors(self):
        return list(self.swap_tensors.values())

    def get_swap_paths(self):
        return list(self.swap_paths.values())

    def get_compute_tensors(self):
        return list(self.compute_tensors.values())

    def get_num_elem(self):
        return self.num_elem


class SwapBufferPool:

    def __init__(self, buffers):
        assert all(b.is_pinned() or not torch.cuda.is_available() for b in buffers)
        self.buffers = [SwapBuffer(b) for b in buffers]
        self.current_index = 0

    def reset(self):
        self.current_index = 0
        for b in self.buffers:
            b.reset()

    def allocate_tensor(self, numel, swap_path, aligned_numel):
        if self.has_space(aligned_numel):
            return self._current().allocate_tensor(swap_path, numel, aligned_numel)
        return None, None

    def insert_tensor(self, tensor, swap_path, aligned_numel):
        if self.has_space(aligned_numel):
            return self._current().insert_tensor(tensor, swap_path, aligned_numel)
        return None, None

    def get_swap_tensors(self):
        return [t for b in self._used() for t in b.get_swap_tensors()]

    def get_swap_paths(self):
        return [p for b in self._used() for p in b.get_swap_paths()]

    def get_compute_tensors(self):
        return [t for b in self._used() for t in b.get_compute_tensors()]

    def has_space(self, numel):
        if self._current().has_space(numel):
            return True
        if self.current_index == len(self.buffers) - 1:
            return False
        self.current_index += 1
        return self._current().has_space(numel)

    def swap_out(self, aio_handle, async_op=False):
        swap_out_tensors(aio_handle, self.get_swap_tensors(), self.get_swap_paths())
        if not async_op:
            assert len(self.get_swap_tensors()) == aio_handle.wait()

    def swap_in(self, aio_handle, async_op=False):
        swap_in_tensors(aio_handle, self.get_swap_tensors(), self.get_swap_paths())
        if not async_op:
            assert len(self.get_swap_tensors()) == aio_handle.wait()

    def _current(self):
        return self.buffers[self.current_index]

    def _used(self):
        return self.buffers[:self.current_index + 1]


class SwapBufferManager:
    """`count` equal slices of one pinned allocation, handed out and returned by index."""

    def __init__(self, num_elems, count, dtype):
        self.num_elems, self.count, self.dtype = num_elems, count, dtype
        from ...accelerator import get_accelerator
        self.all_buffers = [get_accelerator().pin_memory(torch.zeros(num_elems, dtype=dtype)) for _ in range(count)]
        self.free_buffer_index = list(range(count))
        self.used_buffer_index = {}
        self.gigabytes = self.all_buffers[0].element_size() * num_elems * count / 1024**3

    def allocate(self, num_elems, count, dtype):
        assert dtype == self.dtype and num_elems <= self.num_elems
        if count > len(self.free_buffer_index):
            return None
        idx, self.free_buffer_index = self.free_buffer_index[-count:], self.free_buffer_index[:-count]
        out = []
        for i in idx:
            t = self.all_buffers[i].narrow(0, 0, num_elems)
            self.used_buffer_index[id(t)] = i
            out.append(t)
        return out

    def allocate_all(self, num_elems, dtype):
        return self.allocate(num_elems, len(self.free_buffer_index), dtype)

    def free(self, buffers):
        for t in buffers:
            self.free_buffer_index.append(self.used_buffer_index.pop(id(t)))


def get_aligned_numel(numel, element_size, aligned_bytes=AIO_ALIGNED_BYTES):
    per = aligned_bytes // element_size
    return -(-numel // per) * per
