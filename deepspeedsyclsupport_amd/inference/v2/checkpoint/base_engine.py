"""Source of named checkpoint tensors for the inference v2 policies (reference
`inference/v2/checkpoint/base_engine.py`)."""
from abc import ABC, abstractmethod
from typing import Iterable, Tuple

import torch

MEGATRON = "megatron"
HUGGINGFACE = "huggingface"


class CheckpointEngineBase(ABC):
    """Yields (name, tensor) pairs in any order; every tensor of the model exactly once. Names are the
    checkpoint's own: the policy's containers map them."""

    @abstractmethod
    def parameters(self) -> Iterable[Tuple[str, torch.Tensor]]:
        ...
