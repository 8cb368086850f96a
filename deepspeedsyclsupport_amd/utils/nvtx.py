"""roctx ranges around hot framework functions (reference: `deepspeed/utils/nvtx.py:9-19`).

`torch.cuda.nvtx` is backed by roctx on ROCm, so `rocprofv3 --marker-trace` shows ZeRO phases.
"""
import functools

from ..accelerator import get_accelerator


def instrument_w_nvtx(func):

    @functools.wraps(func)
    def wrapped(*args, **kwargs):
        acc = get_accelerator()
        acc.range_push(func.__qualname__)
        try:
            return func(*args, **kwargs)
        finally:
            acc.range_pop()

    return wrapped
