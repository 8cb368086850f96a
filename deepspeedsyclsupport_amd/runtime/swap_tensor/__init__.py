"""ZeRO-Infinity NVMe swapping (reference `runtime/swap_tensor/`)."""
from .optimizer_swapper import OptimizerStateSwapper
from .tensor_swapper import AsyncTensorSwapper
from .param_store import ParamNvmeStore
