"""The MI355X implementations behind the inference v2 module interfaces (reference
`inference/v2/modules/implementations/{attention,embedding,linear,moe,post_norm,pre_norm,unembed}`). Registry names
are the reference's, so a config bundle written for it selects the matching implementation here. Every
implementation is a thin composition of the kernel objects in `inference/v2/kernels`."""
import math
from typing import Any, Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from ....ops import moe_ops
from ....ops.transformer import functional as DF
from ..inference_parameter import InferenceParameter
from ..inference_utils import ActivationType, NormTypeEnum, act_name, is_gated
from ..kernels import (BlockedFlashAttn, BlockedRotaryEmbeddings, BlockedTrainedRotaryEmbeddings, CUDAFPPostLN,
                       CUDAFPPreLN, CUDAFPLN, CUDARMSNorm, CUDARMSPreNorm, LinearBlockedKVCopy, RaggedEmbeddingKernel,
                       RaggedLogitsGather)
from ..kernels.ragged_ops import HEAD_SIZES
from .configs import (DSEmbeddingsConfig, DSLinearConfig, DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                      DSUnembedConfig, MaskingType, PositionalEmbeddingType)
from .interfaces import (DSEmbeddingBase, DSEmbeddingRegistry, DSLinearBase, DSLinearRegistry, DSMoEBase,
                         DSMoERegistry, DSPostNormBase, DSPostNormRegistry, DSPreNormBase, DSPreNormRegistry,
                         DSSelfAttentionBase, DSSelfAttentionRegistry, DSUnembedBase, DSUnembedRegistry)

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`

_FP = (torch.float16, torch.bfloat16, torch.float32)


def _apply_act(x, bias, act: ActivationType):
    act = ActivationType(act)
    if is_gated(act):
        return DF.gated_activation(x if bias is None else x + bias, act_name(act))
    if act == ActivationType.IDENTITY:
        return x if bias is None else x + bias
    return DF.bias_activation(x, bias, act_name(act))


@DSSelfAttentionRegistry.register_module
class DSDenseBlockedAttention(DSSelfAttentionBase):
    """Causal (optionally windowed / ALiBi-biased) attention over the paged KV cache with the rotary variants fused
    into the cache append."""

    @staticmethod
    def name():
        return "dense_blocked_attention"

    @staticmethod
    def supports_config(config: DSSelfAttentionConfig) -> bool:
        if config.input_dtype != config.output_dtype or config.input_dtype.value not in _FP:
            return False
        if config.masking_type not in (MaskingType.causal, MaskingType.local):
            return False
        if config.head_size not in HEAD_SIZES or config.n_heads_q % config.n_heads_kv:
            return False
        pe = config.positional_embedding_type
        if pe in (PositionalEmbeddingType.rotate_half, PositionalEmbeddingType.rotate_every_other):
            return config.positional_embedding_config is not None
        return pe in (PositionalEmbeddingType.none, PositionalEmbeddingType.alibi)

    def __init__(self, config: DSSelfAttentionConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)
        c, dt = config, config.input_dtype.value
        self._interleaved = c.positional_embedding_type == PositionalEmbeddingType.rotate_every_other
        self._trained = False
        if c.positional_embedding_type in (PositionalEmbeddingType.rotate_half,
                                           PositionalEmbeddingType.rotate_every_other):
            rc = c.positional_embedding_config
            if rc.use_trained_freqs:
                self._trained = True
                self._append = BlockedTrainedRotaryEmbeddings(c.head_size, c.n_heads_q, c.n_heads_kv, dt)
            else:
                self._append = BlockedRotaryEmbeddings(c.head_size, c.n_heads_q, c.n_heads_kv, dt,
                                                       rc.rotate_dim or c.head_size, rc.theta_base)
        else:
            self._append = LinearBlockedKVCopy(c.head_size, c.n_heads_q, c.n_heads_kv, dt)
        self._attn = BlockedFlashAttn(c.head_size, dt)
        self._window = int(c.masking_args.get("window_size", 0)) if c.masking_type == MaskingType.local else 0

    @property
    def kv_block_size(self) -> int:
        return 64

    @property
    def q_block_size(self) -> int:
        return 128

    def forward(self, q_k_v: torch.Tensor, kv_cache, batch, attention_mask: Optional[torch.Tensor] = None,
                attention_bias: Optional[torch.Tensor] = None,
                inv_freqs: Optional[torch.Tensor] = None) -> torch.Tensor:
        """q_k_v [tokens, (Hq + 2 Hk) * D]; `attention_bias`: ALiBi slopes [Hq] for PositionalEmbeddingType.alibi.
        Returns [tokens, Hq * D]."""
        c = self._config
        if self._trained:
            q = self._append(kv_cache, q_k_v, batch, inv_freqs)
        elif isinstance(self._append, BlockedRotaryEmbeddings):
            cos, sin = self._append._cos_sin(q_k_v.device, batch.meta.max_len + 1)
            q = self._append._run(kv_cache, q_k_v, batch, cos, sin, self._append.rotary_dim, self._interleaved)
        else:
            q = self._append(kv_cache, q_k_v, batch)
        out = torch.empty(q_k_v.shape[0], c.n_heads_q * c.head_size, dtype=q_k_v.dtype, device=q_k_v.device)
        alibi = attention_bias if c.positional_embedding_type == PositionalEmbeddingType.alibi else None
        return self._attn(out, q, kv_cache, batch, c.scale_factor, alibi, self._window)


@DSEmbeddingRegistry.register_module
class DSRaggedEmbedding(DSEmbeddingBase):

    @staticmethod
    def name():
        return "ragged_embedding"

    @staticmethod
    def supports_config(config: DSEmbeddingsConfig) -> bool:
        return (config.residual_dtype.value in _FP and not config.use_token_type
                and config.output_normalization is None)

    def __init__(self, config: DSEmbeddingsConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)
        self._kernel = RaggedEmbeddingKernel(config.residual_dtype.value, torch.int64, config.embedding_dim)
        self._output = None

    def transform_param(self, embed_param: torch.Tensor) -> InferenceParameter:
        return InferenceParameter.initialize(embed_param.to(self._config.residual_dtype.value))

    @property
    def output(self) -> torch.Tensor:
        return self._output

    def forward(self, ragged_batch, word_embeddings, position_embeddings=None, token_type_ids=None,
                token_type_embeddings=None) -> torch.Tensor:
        out = torch.empty(ragged_batch.current_tokens, self._config.embedding_dim, dtype=word_embeddings.dtype,
                          device=word_embeddings.device)
        self._output = self._kernel(out, ragged_batch, word_embeddings, position_embeddings,
                                    self._config.positional_offset)
        return self._output


@DSLinearRegistry.register_module
class BlasFPLinear(DSLinearBase):
    """Library GEMM + fused bias / activation (gated activations consume 2 x out_channels columns: [gate | up])."""

    @staticmethod
    def name():
        return "blas_fp_linear"

    @staticmethod
    def supports_config(config: DSLinearConfig) -> bool:
        return config.input_dtype == config.output_dtype and config.input_dtype.value in _FP

    def __init__(self, config: DSLinearConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)
        self._output = None

    def transform_param(self, param: torch.Tensor) -> InferenceParameter:
        return InferenceParameter.initialize(param.to(self._config.output_dtype.value))

    @property
    def output(self) -> torch.Tensor:
        return self._output

    def forward(self, hidden_states: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
        act = ActivationType(self._config.activation)
        if act == ActivationType.IDENTITY:
            self._output = F.linear(hidden_states, w, b)
        else:
            self._output = _apply_act(F.linear(hidden_states, w), b, act)
        return self._output


@DSMoERegistry.register_module
class DSMultiGemmMoE(DSMoEBase):
    """Softmax top-k router -> expert-contiguous scatter -> grouped GEMM pair -> weighted gather, without a host
    sync (`ops/moe_ops.moe_block`). Expert weights: mlp_1_w [E, intermediate (x2 when gated), model_dim], mlp_2_w
    [E, model_dim, intermediate]."""

    @staticmethod
    def name():
        return "cutlass_multi_gemm_moe"

    @staticmethod
    def supports_config(config: DSMoEConfig) -> bool:
        return config.input_dtype == config.output_dtype and config.input_dtype.value in _FP and config.top_k >= 1

    def __init__(self, config: DSMoEConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)
        self._output = None

    def _t(self, param):
        return InferenceParameter.initialize(param.to(self._config.input_dtype.value))

    transform_gate_param = transform_moe_mlp_1_param = transform_moe_mlp_2_param = _t

    @property
    def output(self) -> torch.Tensor:
        return self._output

    def forward(self, hidden_states, gate_w, mlp_1_w, mlp_2_w, mlp_1_b=None, mlp_2_b=None) -> torch.Tensor:
        c = self._config
        self._output = moe_ops.moe_block(hidden_states, gate_w, mlp_1_w, mlp_2_w, c.top_k,
                                         lambda h: _apply_act(h, None, c.activation), c.normalize_scores,
                                         fc1_b=mlp_1_b, fc2_b=mlp_2_b)
        return self._output


class _NormParam:

    def transform_param(self, param: torch.Tensor) -> InferenceParameter:
        return InferenceParameter.initialize(param.to(self._config.input_dtype.value))


@DSPreNormRegistry.register_module
class DSPreLNCUDAModule(_NormParam, DSPreNormBase):

    @staticmethod
    def name():
        return "cuda_pre_ln"

    @staticmethod
    def supports_config(config: DSNormConfig) -> bool:
        return (NormTypeEnum(config.type) == NormTypeEnum.LayerNorm and config.input_dtype.value in _FP
                and config.residual_dtype == config.input_dtype == config.output_dtype)

    def __init__(self, config: DSNormConfig, implementation_config: Dict[str, Any]):
        super().__init__(config, implementation_config)
        dt = config.input_dtype.value
        self._first = CUDAFPLN(config.channels, dt, config.eps)
        self._rest = CUDAFPPreLN(config.channels, dt, config.eps)

    def forward(self, residual, hidden_in, gamma, beta=None) -> Tuple[torch.Tensor, torch.Tensor]:
        out = torch.empty_like(residual)
        if hidden_in is None:
            return residual, self._first(out, residual, gamma, beta)
        self._rest(residual, out, residual, hidden_in, gamma, beta)
        return residual, out


@DSPreNormRegistry.register_module
class DSPreRMSCUDAModule(_NormParam, DSPreNormBase):

    @staticmethod
    def name():
        return "cuda_pre_rms"

    @staticmethod
    def supports_config(config: DSNormConfig) -> bool:
        return (NormTypeEnum(config.type) == NormTypeEnum.RMSNorm and config.input_dtype.value in _FP
                and config.residual_dtype == config.input_dtype == config.output_dtype)

    def __init__(self, config: DSNormConfig, implementation_config: Dict[str, Any]):
        super().__init__(config, implementation_config)
        dt = config.input_dtype.value
        self._first = CUDARMSNorm(config.channels, dt, config.eps)
        self._rest = CUDARMSPreNorm(config.channels, dt, config.eps)

    def forward(self, residual, hidden_in, gamma, beta=None) -> Tuple[torch.Tensor, torch.Tensor]:
        out = torch.empty_like(residual)
        if hidden_in is None:
            return residual, self._first(out, residual, gamma)
        self._rest(residual, out, residual, hidden_in, gamma)
        return residual, out


@DSPostNormRegistry.register_module
class DSPostLNCUDAModule(_NormParam, DSPostNormBase):

    @staticmethod
    def name():
        return "cuda_post_ln"

    @staticmethod
    def supports_config(config: DSNormConfig) -> bool:
        return (NormTypeEnum(config.type) == NormTypeEnum.LayerNorm and config.input_dtype.value in _FP
                and config.residual_dtype == config.input_dtype == config.output_dtype)

    def __init__(self, config: DSNormConfig, implementation_config: Dict[str, Any]):
        super().__init__(config, implementation_config)
        self._kernel = CUDAFPPostLN(config.channels, config.input_dtype.value, config.eps)

    def forward(self, residual, hidden_in, gamma, beta) -> torch.Tensor:
        return self._kernel(residual, residual, hidden_in, gamma, beta)


@DSUnembedRegistry.register_module
class DSRaggedUnembed(DSUnembedBase):

    @staticmethod
    def name():
        return "ragged_unembed"

    @staticmethod
    def supports_config(config: DSUnembedConfig) -> bool:
        return config.dtype.value in _FP and config.model_dim % 8 == 0

    def __init__(self, config: DSUnembedConfig, implementation_config: Dict[str, Any]) -> None:
        super().__init__(config, implementation_config)
        self._gather = RaggedLogitsGather(config.model_dim, config.dtype.value)
        self._output = None

    @property
    def output(self) -> torch.Tensor:
        return self._output

    def forward(self, hidden_states, vocab_embedding, ragged_metadata, gamma=None, beta=None) -> torch.Tensor:
        """-> logits [sequences (kernel order), vocab]; `ragged_metadata.restore_order` gives insertion order."""
        c = self._config
        last = torch.empty(ragged_metadata.current_sequences, c.model_dim, dtype=hidden_states.dtype,
                           device=hidden_states.device)
        self._gather(last, hidden_states, ragged_metadata)
        if c.norm_type is not None:
            if NormTypeEnum(c.norm_type) == NormTypeEnum.LayerNorm:
                last = DF.layer_norm(last, gamma, beta, 1e-5)
            else:
                last = DF.rms_norm(last, gamma, 1e-5)
        self._output = F.linear(last, vocab_embedding)
        return self._output


__all__ = ["DSDenseBlockedAttention", "DSRaggedEmbedding", "BlasFPLinear", "DSMultiGemmMoE", "DSPreLNCUDAModule",
           "DSPreRMSCUDAModule", "DSPostLNCUDAModule", "DSRaggedUnembed"]
_ = math
