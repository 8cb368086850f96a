"""Interface configs of the inference v2 modules (reference `inference/v2/modules/configs/*.py`)."""
from enum import Enum
from typing import Dict, Optional

from ..inference_utils import ActivationType, DtypeEnum, NormTypeEnum
from ....runtime.config_utils import DeepSpeedConfigModel
from .ds_module import DSModuleConfig

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`


class PositionalEmbeddingType(Enum):
    none = "none"
    rotate_half = "rotate_half"                  # (x[i], x[i + rot / 2]) pairs (Llama / NeoX)
    rotate_every_other = "rotate_every_other"    # (x[2i], x[2i + 1]) pairs (GPT-J)
    alibi = "alibi"


class RotateHalfConfig(DeepSpeedConfigModel):
    use_trained_freqs: bool = False   # take an `inv_freqs` tensor at call time instead of theta_base
    theta_base: float = 10_000.0
    rotate_dim: Optional[int] = None  # elements of each head that rotate (None: the whole head)


class MaskingType(Enum):
    none = "none"
    causal = "causal"
    local = "local"
    symmetric = "symmetric"
    asymmetric = "asymmetric"


class DSSelfAttentionConfig(DSModuleConfig):
    n_heads_q: int             # query heads on this shard
    n_heads_kv: int            # key / value heads on this shard
    head_size: int
    max_sequences: int
    scale_factor: float = 1.0
    input_dtype: DtypeEnum = DtypeEnum.fp16
    output_dtype: DtypeEnum = DtypeEnum.fp16
    masking_type: MaskingType = MaskingType.causal
    masking_args: Dict = {}    # {"window_size": n} for MaskingType.local
    positional_embedding_type: PositionalEmbeddingType = PositionalEmbeddingType.none
    positional_embedding_config: Optional[RotateHalfConfig] = None


class DSEmbeddingsConfig(DSModuleConfig):
    residual_dtype: DtypeEnum = DtypeEnum.fp16
    embedding_dim: int
    positional_embedding: bool = False
    positional_offset: int = 0           # OPT stores its learned positions shifted by 2
    use_token_type: bool = False
    output_normalization: Optional[NormTypeEnum] = None


class DSLinearConfig(DSModuleConfig):
    in_channels: int
    out_channels: int                    # after the activation: a gated activation consumes 2 x out_channels
    activation: ActivationType = ActivationType.IDENTITY
    input_dtype: DtypeEnum = DtypeEnum.fp16
    output_dtype: DtypeEnum = DtypeEnum.fp16


class DSMoEConfig(DSModuleConfig):
    model_dim: int
    intermediate_features: int
    n_experts: int
    top_k: int = 1
    input_dtype: DtypeEnum = DtypeEnum.fp16
    output_dtype: DtypeEnum = DtypeEnum.fp16
    activation: ActivationType = ActivationType.IDENTITY
    normalize_scores: bool = False


class DSNormConfig(DSModuleConfig):
    type: NormTypeEnum
    channels: int
    residual_dtype: DtypeEnum = DtypeEnum.fp16
    input_dtype: DtypeEnum = DtypeEnum.fp16
    output_dtype: DtypeEnum = DtypeEnum.fp16
    eps: float = 1e-5


class DSUnembedConfig(DSModuleConfig):
    dtype: DtypeEnum = DtypeEnum.fp16
    norm_type: Optional[NormTypeEnum] = None
    model_dim: int
    max_sequences: int
    vocab_size: int
