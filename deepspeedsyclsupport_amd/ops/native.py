"""Access to the in-tree native extensions.

`hip_ops()` returns the gfx950 kernel module. On a machine with a HIP device it MUST load (build errors raise) —
there is no silent eager fallback for device tensors. Host tensors (CPU plumbing path) use the torch reference
implementations in `ops/reference.py` instead, which is the only place non-native math lives.
"""
import functools

import torch

from . import op_builder

DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


@functools.lru_cache(None)
def hip_ops():
    return op_builder.load("ds_hip_ops")


@functools.lru_cache(None)
def cpu_ops():
    return op_builder.load("ds_cpu_ops")


def on_device(t):
    return t.is_cuda


def use_native(*tensors):
    """True when every given tensor lives on the GPU (then the native path is mandatory)."""
    return all(t is None or t.is_cuda for t in tensors) and any(t is not None and t.is_cuda for t in tensors)
