"""Base class of the inference v2 kernel objects (reference `inference/v2/kernels/ds_kernel.py`): constructed once
per configuration (validating dtypes / sizes up front), then called per forward."""
from abc import ABC, abstractmethod


class DSKernelBase(ABC):

    @abstractmethod
    def __init__(self, *args, **kwargs):
        raise NotImplementedError()

    @abstractmethod
    def __call__(self, *args, **kwargs):
        raise NotImplementedError()
