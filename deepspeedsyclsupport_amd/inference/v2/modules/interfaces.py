"""Interfaces and registries of the inference v2 modules (reference `inference/v2/modules/interfaces/*.py`): one
abstract base per building block and the registry its implementations sign up to."""
from typing import Any, Dict, Optional, Tuple, Type

import torch

from ..inference_parameter import InferenceParameter
from .configs import (DSEmbeddingsConfig, DSLinearConfig, DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                      DSUnembedConfig)
from .ds_module import DSModuleBase
from .module_registry import DSModuleRegistryBase

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`


def _registry(interface):

    class _Registry(DSModuleRegistryBase):
        registry: Dict = {}

        @staticmethod
        def associated_class() -> Type[DSModuleBase]:
            return interface

    _Registry.__name__ = _Registry.__qualname__ = interface.__name__.replace("Base", "Registry")
    return _Registry


class DSSelfAttentionBase(DSModuleBase):
    """qkv of every token of a ragged batch -> attention output; appends k / v to the paged cache on the way."""

    @staticmethod
    def config_class():
        return DSSelfAttentionConfig

    def __init__(self, config: DSSelfAttentionConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)

    @property
    def kv_block_size(self) -> int:
        raise NotImplementedError()

    @property
    def q_block_size(self) -> int:
        raise NotImplementedError()

    def build_atoms(self, ragged_batch) -> None:
        pass

    def forward(self, q_k_v: torch.Tensor, kv_cache, batch, attention_mask: Optional[torch.Tensor] = None,
                attention_bias: Optional[torch.Tensor] = None,
                inv_freqs: Optional[torch.Tensor] = None) -> torch.Tensor:
        raise NotImplementedError()


class DSEmbeddingBase(DSModuleBase):
    """Token ids of a ragged batch -> embedded hidden states (word + optional position / token-type tables)."""

    @staticmethod
    def config_class():
        return DSEmbeddingsConfig

    def __init__(self, config: DSEmbeddingsConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)

    def transform_param(self, embed_param: torch.Tensor) -> InferenceParameter:
        raise NotImplementedError()

    @property
    def output(self) -> torch.Tensor:
        raise NotImplementedError()

    def forward(self, ragged_batch, word_embeddings: torch.Tensor, position_embeddings: Optional[torch.Tensor] = None,
                token_type_ids: Optional[torch.Tensor] = None,
                token_type_embeddings: Optional[torch.Tensor] = None) -> torch.Tensor:
        raise NotImplementedError()


class DSLinearBase(DSModuleBase):
    """activation(hidden_states . w^T + b); `transform_param` converts a checkpoint weight to what forward takes."""

    @staticmethod
    def config_class():
        return DSLinearConfig

    def __init__(self, config: DSLinearConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)

    def transform_param(self, param: torch.Tensor) -> InferenceParameter:
        raise NotImplementedError()

    def forward(self, hidden_states: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
        raise NotImplementedError()

    @property
    def output(self) -> torch.Tensor:
        raise NotImplementedError()


class DSMoEBase(DSModuleBase):
    """Top-k routed expert MLP."""

    @staticmethod
    def config_class():
        return DSMoEConfig

    def __init__(self, config: DSMoEConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)

    def transform_gate_param(self, param: torch.Tensor) -> InferenceParameter:
        raise NotImplementedError()

    def transform_moe_mlp_1_param(self, param: torch.Tensor) -> InferenceParameter:
        raise NotImplementedError()

    def transform_moe_mlp_2_param(self, param: torch.Tensor) -> InferenceParameter:
        raise NotImplementedError()

    def forward(self, hidden_states: torch.Tensor, gate_w: torch.Tensor, mlp_1_w: torch.Tensor,
                mlp_2_w: torch.Tensor, mlp_1_b: Optional[torch.Tensor] = None,
                mlp_2_b: Optional[torch.Tensor] = None) -> torch.Tensor:
        raise NotImplementedError()

    @property
    def output(self) -> torch.Tensor:
        raise NotImplementedError()


class DSPreNormBase(DSModuleBase):
    """residual += hidden_states (if given); hidden_states = norm(residual). Returns (residual, hidden_states)."""

    @staticmethod
    def config_class():
        return DSNormConfig

    def __init__(self, config: DSNormConfig, implementation_config: Dict[str, Any]):
        super().__init__(config, implementation_config)

    def transform_param(self, param: torch.Tensor) -> InferenceParameter:
        raise NotImplementedError()

    def forward(self, residual: torch.Tensor, hidden_states: Optional[torch.Tensor], gamma: torch.Tensor,
                beta: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        raise NotImplementedError()


class DSPostNormBase(DSModuleBase):
    """residual = norm(residual + hidden_states). Returns the new residual."""

    @staticmethod
    def config_class():
        return DSNormConfig

    def __init__(self, config: DSNormConfig, implementation_config: Dict[str, Any]):
        super().__init__(config, implementation_config)

    def transform_param(self, param: torch.Tensor) -> InferenceParameter:
        raise NotImplementedError()

    def forward(self, residual: torch.Tensor, hidden_states: torch.Tensor, gamma: torch.Tensor,
                beta: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError()


class DSUnembedBase(DSModuleBase):
    """Final-token hidden states (optionally normalised) -> logits [sequences, vocab]."""

    @staticmethod
    def config_class():
        return DSUnembedConfig

    def __init__(self, config: DSUnembedConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)

    def forward(self, hidden_states: torch.Tensor, vocab_embedding: torch.Tensor, ragged_metadata,
                gamma: Optional[torch.Tensor] = None, beta: Optional[torch.Tensor] = None) -> torch.Tensor:
        raise NotImplementedError()


DSSelfAttentionRegistry = _registry(DSSelfAttentionBase)
DSEmbeddingRegistry = _registry(DSEmbeddingBase)
DSLinearRegistry = _registry(DSLinearBase)
DSMoERegistry = _registry(DSMoEBase)
DSPreNormRegistry = _registry(DSPreNormBase)
DSPostNormRegistry = _registry(DSPostNormBase)
DSUnembedRegistry = _registry(DSUnembedBase)
