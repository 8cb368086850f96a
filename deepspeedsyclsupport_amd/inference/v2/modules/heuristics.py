"""Choice of implementation per building block (reference `inference/v2/modules/heuristics.py`): a model asks for "an
attention / linear / norm for this config" and gets the registered implementation that fits this engine."""
from .configs import (DSEmbeddingsConfig, DSLinearConfig, DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                      DSUnembedConfig)
from ..inference_utils import NormTypeEnum
from . import implementations  # noqa: F401  (registers the implementations)
from .interfaces import (DSEmbeddingRegistry, DSLinearRegistry, DSMoERegistry, DSPostNormRegistry, DSPreNormRegistry,
                         DSSelfAttentionRegistry, DSUnembedRegistry)
from .module_registry import ConfigBundle


def instantiate_attention(attention_config: DSSelfAttentionConfig, engine_config=None):
    return DSSelfAttentionRegistry.instantiate_config(
        ConfigBundle(name="dense_blocked_attention", config=attention_config))


def instantiate_embed(embed_config: DSEmbeddingsConfig, engine_config=None):
    return DSEmbeddingRegistry.instantiate_config(ConfigBundle(name="ragged_embedding", config=embed_config))


def instantiate_linear(linear_config: DSLinearConfig, engine_config=None):
    return DSLinearRegistry.instantiate_config(ConfigBundle(name="blas_fp_linear", config=linear_config))


def instantiate_moe(moe_config: DSMoEConfig, engine_config=None):
    return DSMoERegistry.instantiate_config(ConfigBundle(name="cutlass_multi_gemm_moe", config=moe_config,
                                                         implementation_config={"weight_dtype":
                                                                                moe_config.input_dtype}))


def instantiate_post_norm(norm_config: DSNormConfig, engine_config=None):
    return DSPostNormRegistry.instantiate_config(ConfigBundle(name="cuda_post_ln", config=norm_config))


def instantiate_pre_norm(norm_config: DSNormConfig, engine_config=None):
    name = "cuda_pre_rms" if NormTypeEnum(norm_config.type) == NormTypeEnum.RMSNorm else "cuda_pre_ln"
    return DSPreNormRegistry.instantiate_config(ConfigBundle(name=name, config=norm_config))


def instantiate_unembed(unembed_config: DSUnembedConfig, engine_config=None):
    return DSUnembedRegistry.instantiate_config(ConfigBundle(name="ragged_unembed", config=unembed_config))
