"""Async tensor I/O front-end (reference `ops/aio`: `AsyncIOBuilder().load().aio_handle(...)`): the native thread
pool with O_DIRECT reads / writes of pinned host tensors (`csrc/cpu/aio.cpp`) that the ZeRO-Infinity swappers use."""
from ..op_builder import AsyncIOBuilder  # noqa: F401


def aio_handle(block_size=1 << 20, queue_depth=8, single_submit=False, overlap_events=True, num_threads=1,
               thread_count=None):
    from ..native import cpu_ops
    return cpu_ops().aio_handle(block_size, queue_depth, single_submit, overlap_events,
                                thread_count if thread_count is not None else num_threads)
