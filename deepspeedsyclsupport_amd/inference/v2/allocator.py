"""Allocation helpers of the ragged engine (reference `inference/v2/allocator.py`)."""
from functools import reduce
from typing import Iterable

import torch

from ...accelerator import get_accelerator


def on_device(method):
    """Decorator: the wrapped function's tensor result (or every tensor of a tuple / list result) is moved to the
    current accelerator device."""

    def wrapped(self, *args, **kwargs):
        dev = get_accelerator().current_device_name()
        out = method(self, *args, **kwargs)
        if isinstance(out, torch.Tensor):
            return out.to(dev)
        if isinstance(out, (tuple, list)):
            return type(out)(o.to(dev) if isinstance(o, torch.Tensor) else o for o in out)
        return out

    return wrapped


def empty_from(tensor: torch.Tensor, shape: Iterable[int]) -> torch.Tensor:
    """A view of `shape` over the leading elements of `tensor` (a preallocated scratch buffer): no allocation."""
    shape = tuple(shape)
    n = reduce(lambda a, b: a * b, shape, 1)
    if n > tensor.numel():
        raise ValueError(f"a view of {shape} needs {n} elements, the buffer holds {tensor.numel()}")
    return tensor.flatten()[:n].view(shape)
