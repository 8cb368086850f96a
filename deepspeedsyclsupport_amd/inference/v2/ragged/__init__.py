"""Ragged-batch state of the inference v2 engine (reference `inference/v2/ragged/`)."""
from ...kv_cache import BlockedAllocator, BlockedKVCache
from .ragged_manager import DSStateManager
from .ragged_wrapper import RaggedBatchWrapper, to_padded
from .sequence_descriptor import BaseSequenceDescriptor, DSSequenceDescriptor, PlaceholderSequenceDescriptor

__all__ = ["BlockedAllocator", "BlockedKVCache", "DSStateManager", "RaggedBatchWrapper", "to_padded",
           "BaseSequenceDescriptor", "DSSequenceDescriptor", "PlaceholderSequenceDescriptor"]
