"""What the ragged engine needs from a model (reference
`inference/v2/model_implementations/inference_model_base.py`, `inference_transformer_base.py`).

In this framework every supported architecture is one configurable implementation,
`inference/model_implementations/transformer.py: DSInferenceModel`, described by a `DSModelSpec`; the reference's
per-architecture model classes (`Llama2InferenceModel`, ...) are thin subclasses of it that pin the architecture
name. `DSInferenceModelBase` states the protocol for models written from the building blocks of
`inference/v2/modules` instead.
"""
from abc import ABC, abstractmethod
from enum import Enum

import torch


class MPType(Enum):
    """How a tensor is laid out across tensor-parallel ranks."""
    REPLICATED = 0
    SHARDED_OUTER = 1
    SHARDED_INNER = 2


class DSInferenceModelBase(torch.nn.Module, ABC):
    """Protocol used by `InferenceEngineV2`: `spec` (layer / head counts for KV sizing), `tp_size`, `tp_rank`,
    `dtype`, `device`, `allocate_cache(num_blocks, block_size)` and `forward_ragged(token_ids, meta)` returning one
    row of logits per sequence in kernel order."""

    @abstractmethod
    def allocate_cache(self, num_blocks: int, block_size: int) -> None:
        ...

    @abstractmethod
    def forward_ragged(self, tokens: torch.Tensor, meta) -> torch.Tensor:
        ...

    def get_kv_requirements(self, sequence, max_new_tokens: int, max_new_blocks: int):
        """(tokens that fit, blocks they need) for a sequence descriptor."""
        n = max_new_tokens
        while n > 0 and sequence.blocks_needed(n) > max_new_blocks:
            n -= 1
        return n, sequence.blocks_needed(n)

    def maybe_allocate_kv(self, sequence, n_new_tokens: int, allocator) -> None:
        need = sequence.blocks_needed(n_new_tokens)
        if need:
            sequence.extend_kv_cache(allocator.allocate(need))

    def maybe_free_kv(self, sequence) -> None:
        """Sliding-window models could return blocks that fell out of the window; dense attention keeps all."""
        return None
