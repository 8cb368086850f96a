"""Ragged-batching (FastGen-style) inference engine."""
from .config_v2 import RaggedInferenceEngineConfig, DSStateManagerConfig, MemoryConfig, AllocationMode, KVCacheConfig
from .engine_factory import build_engine_from_ds_checkpoint, build_hf_engine
from .engine_v2 import InferenceEngineV2
from .scheduling_utils import SchedulingError, SchedulingResult
