"""Configurable building blocks of inference v2 (reference `inference/v2/modules/`)."""
from . import implementations
from .configs import (DSEmbeddingsConfig, DSLinearConfig, DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                      DSUnembedConfig, MaskingType, PositionalEmbeddingType, RotateHalfConfig)
from .ds_module import DSModuleBase, DSModuleConfig
from .heuristics import (instantiate_attention, instantiate_embed, instantiate_linear, instantiate_moe,
                         instantiate_post_norm, instantiate_pre_norm, instantiate_unembed)
from .module_registry import ConfigBundle, DSModuleRegistryBase
