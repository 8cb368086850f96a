"""Asynchronous tensor <-> file swapping on the native thread-pool aio engine (reference
`runtime/swap_tensor/async_swapper.py:19`, `utils.py` swap_in_tensors / swap_out_tensors)."""
import os

import torch


def _aio(aio_config):
    from ...ops.native import cpu_ops
    c = aio_config
    return cpu_ops().aio_handle(c.block_size, c.queue_depth, c.single_submit, c.overlap_events, c.thread_count)


class AsyncTensorSwapper:
    """Separate read / write handles so a write-back never stalls the next prefetch."""

    def __init__(self, aio_config, folder):
        os.makedirs(folder, exist_ok=True)
        self.folder = folder
        self.reader = _aio(aio_config)
        self.writer = _aio(aio_config)

    def path(self, key):
        return os.path.join(self.folder, f"{key}.tensor.swp")

    def swap_out(self, key, tensor, async_op=True):
        t = tensor if tensor.is_contiguous() else tensor.contiguous()
        if async_op:
            self.writer.async_pwrite(t, self.path(key))
        else:
            self.writer.sync_pwrite(t, self.path(key))

    def swap_in(self, key, buffer, async_op=True):
        if async_op:
            self.reader.async_pread(buffer, self.path(key))
        else:
            self.reader.sync_pread(buffer, self.path(key))

    def wait_reads(self):
        return self.reader.wait()

    def wait_writes(self):
        return self.writer.wait()

    def exists(self, key):
        return os.path.exists(self.path(key))
