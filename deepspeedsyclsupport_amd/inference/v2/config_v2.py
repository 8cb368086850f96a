"""Ragged (FastGen-style) engine configuration (reference `inference/v2/config_v2.py`, `ragged/manager_configs.py`)."""
from enum import Enum
from typing import Optional

from pydantic import PositiveInt, model_validator

from ...runtime.config_utils import DeepSpeedConfigModel
from ..config import DeepSpeedTPConfig


class AllocationMode(Enum):
    RESERVE = "reserve"      # size = bytes of HBM to leave free after sizing the KV cache
    ALLOCATE = "allocate"    # size = number of KV blocks


class MemoryConfig(DeepSpeedConfigModel):
    mode: AllocationMode = AllocationMode.RESERVE
    size: PositiveInt = 1_000_000_000


class KVCacheConfig(DeepSpeedConfigModel):
    block_size: int = 64   # tokens per block (64 x head_dim x 2 B = one 16 KB contiguous K slab per head at D=128)


class DSStateManagerConfig(DeepSpeedConfigModel):
    max_tracked_sequences: PositiveInt = 2048
    max_ragged_batch_size: PositiveInt = 768
    max_ragged_sequence_count: PositiveInt = 512
    max_context: PositiveInt = 8192
    memory_config: MemoryConfig = MemoryConfig()
    offload: bool = False

    @model_validator(mode="after")
    def _check(self):
        if self.max_ragged_sequence_count > self.max_tracked_sequences:
            raise ValueError("max_ragged_sequence_count must be <= max_tracked_sequences")
        if self.max_ragged_sequence_count > self.max_ragged_batch_size:
            raise ValueError("max_ragged_sequence_count must be <= max_ragged_batch_size")
        return self


class QuantizationConfig(DeepSpeedConfigModel):
    quantization_mode: Optional[str] = None   # None | "int8" | "int4" (weight-only)


class RaggedInferenceEngineConfig(DeepSpeedConfigModel):
    tensor_parallel: DeepSpeedTPConfig = DeepSpeedTPConfig()
    state_manager: DSStateManagerConfig = DSStateManagerConfig()
    kv_cache: KVCacheConfig = KVCacheConfig()
    quantization: QuantizationConfig = QuantizationConfig()
    enable_cuda_graph: bool = False
    # bf16 projection weights for small ragged batches (<= 16 tokens), see `DeepSpeedInferenceConfig.decode_layout`
    decode_layout: str = "auto"
