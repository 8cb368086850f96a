"""Containers, policies and model classes of the architectures served by the ragged engine (reference
`inference/v2/model_implementations/{llama_v2,mistral,mixtral,opt,phi,falcon}/{container,policy,model}.py`).

Mapping keys are the tensor names of the Hugging Face checkpoints; the parameter classes turn them into canonical
layer entries (`common_parameters.py`).
"""
from ...model_implementations.transformer import DSInferenceModel
from .common_parameters import (AttentionOutputParameter, EmbeddingParameter, FusedMoEGatedMLPParameter,
                                FusedMoEMLP2Parameter, FusedQKVBias, FusedQKVParameter, GatedMLPParameter,
                                GQAMegatronQKVParameter, MegatronQKVParameter, MLP1Parameter, MLP2Parameter,
                                MoEGatingWeightParameter, NormParameter, UnembedParameter, UnfusedMoEGatedMLPParameter,
                                UnfusedMoEMLP2Parameter, UnfusedQKVBias, UnfusedQKVParameter)
from .inference_policy_base import ContainerMap, InferenceV2Policy, register
from .layer_container_base import LayerContainer


def _opt(cls):
    """The same parameter type, allowed to stay empty (an absent bias / a checkpoint variant)."""
    return type(cls.__name__ + "Optional", (cls, ), {"optional": True, "__annotations__": {}})


def _model_class(name, arch_doc):
    cls = type(name, (DSInferenceModel, ), {"__doc__": f"{arch_doc} on the ragged engine: `DSInferenceModel` with "
                                                       f"the spec its policy derives from the HF config."})
    return cls


# ------------------------------------------------------------------------------------------------ Llama-2 / Mistral
class Llama2TransformerContainer(LayerContainer):
    qkv_w: UnfusedQKVParameter
    qkv_b: _opt(UnfusedQKVBias)
    attn_out_w: AttentionOutputParameter.as_("o_w")
    mlp_1_w: GatedMLPParameter
    mlp_2_w: MLP2Parameter.as_("fc2_w")
    attn_norm_gamma: NormParameter.as_("ln1_w")
    mlp_norm_gamma: NormParameter.as_("ln2_w")

    PARAM_MAPPING = {
        "self_attn.q_proj.weight": "qkv_w.q_params",
        "self_attn.k_proj.weight": "qkv_w.k_params",
        "self_attn.v_proj.weight": "qkv_w.v_params",
        "self_attn.q_proj.bias": "qkv_b.q_params",
        "self_attn.k_proj.bias": "qkv_b.k_params",
        "self_attn.v_proj.bias": "qkv_b.v_params",
        "self_attn.o_proj.weight": "attn_out_w.params",
        "mlp.gate_proj.weight": "mlp_1_w.gate_params",
        "mlp.up_proj.weight": "mlp_1_w.up_params",
        "mlp.down_proj.weight": "mlp_2_w.params",
        "input_layernorm.weight": "attn_norm_gamma.params",
        "post_attention_layernorm.weight": "mlp_norm_gamma.params",
    }


class Llama2NonTransformerContainer(LayerContainer):
    word_emb: EmbeddingParameter
    word_unembed: _opt(UnembedParameter)
    final_norm: NormParameter.as_("norm_w")

    PARAM_MAPPING = {
        "model.embed_tokens.weight": "word_emb.params",
        "model.norm.weight": "final_norm.params",
        "lm_head.weight": "word_unembed.params",
    }


class _DecoderPolicy(InferenceV2Policy):
    layer_prefix = "model.layers"
    transformer_container = None
    non_transformer_container = None
    unmapped = (r"rotary_emb\.inv_freq$", r"\.masked_bias$", r"\.attn\.bias$")

    def build_container_map(self) -> ContainerMap:
        cmap = ContainerMap()
        view = self._view
        cmap.set_transformer_params(self.layer_prefix, [self.transformer_container(view)
                                                        for _ in range(view.spec.num_layers)])
        cmap.set_non_transformer_params(self.non_transformer_container(view))
        cmap.set_unmapped_params(self.unmapped)
        return cmap


Llama2InferenceModel = _model_class("Llama2InferenceModel", "Llama-2")
MistralInferenceModel = _model_class("MistralInferenceModel", "Mistral (sliding-window Llama stack)")
MistralTransformerContainer = Llama2TransformerContainer
MistralNonTransformerContainer = Llama2NonTransformerContainer


@register
class Llama2Policy(_DecoderPolicy):
    model_types = ("llama", )
    transformer_container = Llama2TransformerContainer
    non_transformer_container = Llama2NonTransformerContainer


@register
class MistralPolicy(_DecoderPolicy):
    model_types = ("mistral", "qwen2")
    transformer_container = Llama2TransformerContainer
    non_transformer_container = Llama2NonTransformerContainer


# ------------------------------------------------------------------------------------------------ Mixtral
class MixtralTransformerContainer(LayerContainer):
    """Accepts both on-disk expert layouts: per-expert w1 / w3 / w2 matrices, or experts stacked as gate_up_proj /
    down_proj."""
    qkv_w: UnfusedQKVParameter
    attn_out_w: AttentionOutputParameter.as_("o_w")
    moe_gate: MoEGatingWeightParameter
    moe_mlp_1: _opt(UnfusedMoEGatedMLPParameter)
    moe_mlp_2: _opt(UnfusedMoEMLP2Parameter)
    moe_fused_1: _opt(FusedMoEGatedMLPParameter)
    moe_fused_2: _opt(FusedMoEMLP2Parameter)
    attn_norm_gamma: NormParameter.as_("ln1_w")
    mlp_norm_gamma: NormParameter.as_("ln2_w")

    PARAM_MAPPING = {
        "input_layernorm.weight": "attn_norm_gamma.params",
        "post_attention_layernorm.weight": "mlp_norm_gamma.params",
        "self_attn.q_proj.weight": "qkv_w.q_params",
        "self_attn.k_proj.weight": "qkv_w.k_params",
        "self_attn.v_proj.weight": "qkv_w.v_params",
        "self_attn.o_proj.weight": "attn_out_w.params",
        "block_sparse_moe.gate.weight": "moe_gate.params",
        "block_sparse_moe.experts.*.w1.weight": "moe_mlp_1.gating_experts",
        "block_sparse_moe.experts.*.w3.weight": "moe_mlp_1.up_experts",
        "block_sparse_moe.experts.*.w2.weight": "moe_mlp_2.experts",
        "mlp.gate.weight": "moe_gate.params",
        "mlp.experts.gate_up_proj": "moe_fused_1.params",
        "mlp.experts.down_proj": "moe_fused_2.params",
    }


MixtralNonTransformerContainer = Llama2NonTransformerContainer
MixtralInferenceModel = _model_class("MixtralInferenceModel", "Mixtral (top-k routed gated experts)")


@register
class MixtralPolicy(_DecoderPolicy):
    model_types = ("mixtral", )
    transformer_container = MixtralTransformerContainer
    non_transformer_container = Llama2NonTransformerContainer

    def _layer_done(self, c) -> bool:
        p = c._params
        core = all(p[n].complete for n in ("qkv_w", "attn_out_w", "moe_gate", "attn_norm_gamma", "mlp_norm_gamma"))
        return core and ((p["moe_mlp_1"].complete and p["moe_mlp_2"].complete)
                         or (p["moe_fused_1"].complete and p["moe_fused_2"].complete))


# ------------------------------------------------------------------------------------------------ OPT
class OPTTransformerContainer(LayerContainer):
    qkv_w: UnfusedQKVParameter
    qkv_b: UnfusedQKVBias
    attn_out_w: AttentionOutputParameter.as_("o_w")
    attn_out_b: AttentionOutputParameter.as_("o_b")
    mlp_1_w: MLP1Parameter.as_("fc1_w")
    mlp_1_b: MLP1Parameter.as_("fc1_b")
    mlp_2_w: MLP2Parameter.as_("fc2_w")
    mlp_2_b: MLP2Parameter.as_("fc2_b")
    attn_norm_gamma: NormParameter.as_("ln1_w")
    attn_norm_beta: NormParameter.as_("ln1_b")
    mlp_norm_gamma: NormParameter.as_("ln2_w")
    mlp_norm_beta: NormParameter.as_("ln2_b")

    PARAM_MAPPING = {
        "self_attn.q_proj.weight": "qkv_w.q_params",
        "self_attn.q_proj.bias": "qkv_b.q_params",
        "self_attn.k_proj.weight": "qkv_w.k_params",
        "self_attn.k_proj.bias": "qkv_b.k_params",
        "self_attn.v_proj.weight": "qkv_w.v_params",
        "self_attn.v_proj.bias": "qkv_b.v_params",
        "self_attn.out_proj.weight": "attn_out_w.params",
        "self_attn.out_proj.bias": "attn_out_b.params",
        "fc1.weight": "mlp_1_w.params",
        "fc1.bias": "mlp_1_b.params",
        "fc2.weight": "mlp_2_w.params",
        "fc2.bias": "mlp_2_b.params",
        "self_attn_layer_norm.weight": "attn_norm_gamma.params",
        "self_attn_layer_norm.bias": "attn_norm_beta.params",
        "final_layer_norm.weight": "mlp_norm_gamma.params",
        "final_layer_norm.bias": "mlp_norm_beta.params",
    }


class OPTNonTransformerContainer(LayerContainer):
    word_emb: EmbeddingParameter
    word_unembed: _opt(UnembedParameter)
    word_emb_pos: NormParameter.as_("pos_embed")
    final_norm_w: NormParameter.as_("norm_w")
    final_norm_b: NormParameter.as_("norm_b")

    PARAM_MAPPING = {
        "*decoder.embed_tokens.weight": "word_emb.params",
        "*decoder.embed_positions.weight": "word_emb_pos.params",
        "*decoder.final_layer_norm.weight": "final_norm_w.params",
        "*decoder.final_layer_norm.bias": "final_norm_b.params",
        "lm_head.weight": "word_unembed.params",
    }


OPTInferenceModel = _model_class("OPTInferenceModel", "OPT (learned positions offset by 2, ReLU MLP)")


@register
class OPTPolicy(_DecoderPolicy):
    model_types = ("opt", )
    layer_prefix = ("model.decoder.layers", "decoder.layers")
    transformer_container = OPTTransformerContainer
    non_transformer_container = OPTNonTransformerContainer


# ------------------------------------------------------------------------------------------------ Phi
class PhiTransformerContainer(LayerContainer):
    """Phi-1 / 1.5 / 2 in the transformers layout (separate q / k / v, `dense`, `fc1` / `fc2`, one LayerNorm) or the
    original `mixer.Wqkv` layout."""
    qkv_w: _opt(UnfusedQKVParameter)
    qkv_b: _opt(UnfusedQKVBias)
    fused_qkv_w: _opt(FusedQKVParameter)
    fused_qkv_b: _opt(FusedQKVBias)
    attn_out_w: AttentionOutputParameter.as_("o_w")
    attn_out_b: AttentionOutputParameter.as_("o_b")
    mlp_1_w: MLP1Parameter.as_("fc1_w")
    mlp_1_b: MLP1Parameter.as_("fc1_b")
    mlp_2_w: MLP2Parameter.as_("fc2_w")
    mlp_2_b: MLP2Parameter.as_("fc2_b")
    ln_gamma: NormParameter.as_("ln1_w")
    ln_beta: NormParameter.as_("ln1_b")

    PARAM_MAPPING = {
        "self_attn.q_proj.weight": "qkv_w.q_params",
        "self_attn.k_proj.weight": "qkv_w.k_params",
        "self_attn.v_proj.weight": "qkv_w.v_params",
        "self_attn.q_proj.bias": "qkv_b.q_params",
        "self_attn.k_proj.bias": "qkv_b.k_params",
        "self_attn.v_proj.bias": "qkv_b.v_params",
        "self_attn.dense.weight": "attn_out_w.params",
        "self_attn.dense.bias": "attn_out_b.params",
        "input_layernorm.weight": "ln_gamma.params",
        "input_layernorm.bias": "ln_beta.params",
        "mixer.Wqkv.weight": "fused_qkv_w.params",
        "mixer.Wqkv.bias": "fused_qkv_b.params",
        "mixer.out_proj.weight": "attn_out_w.params",
        "mixer.out_proj.bias": "attn_out_b.params",
        "ln.weight": "ln_gamma.params",
        "ln.bias": "ln_beta.params",
        "mlp.fc1.weight": "mlp_1_w.params",
        "mlp.fc1.bias": "mlp_1_b.params",
        "mlp.fc2.weight": "mlp_2_w.params",
        "mlp.fc2.bias": "mlp_2_b.params",
    }


class PhiNonTransformerContainer(LayerContainer):
    word_emb: EmbeddingParameter
    word_unembed_w: UnembedParameter
    word_unembed_b: NormParameter.as_("lm_head_b")
    final_norm_gamma: NormParameter.as_("norm_w")
    final_norm_beta: NormParameter.as_("norm_b")

    PARAM_MAPPING = {
        "model.embed_tokens.weight": "word_emb.params",
        "model.final_layernorm.weight": "final_norm_gamma.params",
        "model.final_layernorm.bias": "final_norm_beta.params",
        "lm_head.weight": "word_unembed_w.params",
        "lm_head.bias": "word_unembed_b.params",
        "transformer.embd.wte.weight": "word_emb.params",
        "lm_head.ln.weight": "final_norm_gamma.params",
        "lm_head.ln.bias": "final_norm_beta.params",
        "lm_head.linear.weight": "word_unembed_w.params",
        "lm_head.linear.bias": "word_unembed_b.params",
    }


PhiInferenceModel = _model_class("PhiInferenceModel", "Phi (parallel block, partial rotary)")


@register
class PhiPolicy(_DecoderPolicy):
    model_types = ("phi", )
    layer_prefix = ("model.layers", "transformer.h")
    transformer_container = PhiTransformerContainer
    non_transformer_container = PhiNonTransformerContainer

    def _layer_done(self, c) -> bool:
        p = c._params
        rest = all(p[n].complete for n in ("attn_out_w", "attn_out_b", "mlp_1_w", "mlp_1_b", "mlp_2_w", "mlp_2_b",
                                           "ln_gamma", "ln_beta"))
        return rest and ((p["qkv_w"].complete and p["qkv_b"].complete)
                         or (p["fused_qkv_w"].complete and p["fused_qkv_b"].complete))


# ------------------------------------------------------------------------------------------------ Falcon
class FalconTransformerContainer(LayerContainer):
    """Falcon-7B style: one LayerNorm, multi-query fused QKV [q heads | k | v]."""
    qkv_w: FusedQKVParameter
    attn_out_w: AttentionOutputParameter.as_("o_w")
    mlp_1_w: MLP1Parameter.as_("fc1_w")
    mlp_2_w: MLP2Parameter.as_("fc2_w")
    ln_attn_gamma: NormParameter.as_("ln1_w")
    ln_attn_beta: NormParameter.as_("ln1_b")

    PARAM_MAPPING = {
        "self_attention.query_key_value.weight": "qkv_w.params",
        "self_attention.dense.weight": "attn_out_w.params",
        "mlp.dense_h_to_4h.weight": "mlp_1_w.params",
        "mlp.dense_4h_to_h.weight": "mlp_2_w.params",
        "input_layernorm.weight": "ln_attn_gamma.params",
        "input_layernorm.bias": "ln_attn_beta.params",
    }


class FalconMHATransformerContainer(FalconTransformerContainer):
    """Falcon without multi-query: per-head interleaved fused QKV."""
    qkv_w: MegatronQKVParameter


class FalconNewArchTransformerContainer(LayerContainer):
    """Falcon-40B / 180B: grouped fused QKV, separate attention / MLP LayerNorms."""
    qkv_w: GQAMegatronQKVParameter
    attn_out_w: AttentionOutputParameter.as_("o_w")
    mlp_1_w: MLP1Parameter.as_("fc1_w")
    mlp_2_w: MLP2Parameter.as_("fc2_w")
    ln_attn_gamma: NormParameter.as_("ln1_w")
    ln_attn_beta: NormParameter.as_("ln1_b")
    ln_mlp_gamma: NormParameter.as_("ln2_w")
    ln_mlp_beta: NormParameter.as_("ln2_b")

    PARAM_MAPPING = {
        "self_attention.query_key_value.weight": "qkv_w.params",
        "self_attention.dense.weight": "attn_out_w.params",
        "mlp.dense_h_to_4h.weight": "mlp_1_w.params",
        "mlp.dense_4h_to_h.weight": "mlp_2_w.params",
        "ln_attn.weight": "ln_attn_gamma.params",
        "ln_attn.bias": "ln_attn_beta.params",
        "ln_mlp.weight": "ln_mlp_gamma.params",
        "ln_mlp.bias": "ln_mlp_beta.params",
    }


class FalconNonTransformerContainer(LayerContainer):
    word_emb: EmbeddingParameter
    word_unembed: _opt(UnembedParameter)
    final_norm_gamma: NormParameter.as_("norm_w")
    final_norm_beta: NormParameter.as_("norm_b")

    PARAM_MAPPING = {
        "transformer.word_embeddings.weight": "word_emb.params",
        "transformer.ln_f.weight": "final_norm_gamma.params",
        "transformer.ln_f.bias": "final_norm_beta.params",
        "lm_head.weight": "word_unembed.params",
    }


FalconInferenceModel = _model_class("FalconInferenceModel", "Falcon (parallel attention + MLP, multi-query)")


@register
class FalconPolicy(_DecoderPolicy):
    model_types = ("falcon", )
    layer_prefix = "transformer.h"
    non_transformer_container = FalconNonTransformerContainer

    @property
    def transformer_container(self):
        cfg = self._model_config
        if cfg.new_decoder_architecture:
            if (cfg.num_ln_in_parallel_attn or 2) == 2:
                return FalconNewArchTransformerContainer
            return type("FalconNewArchOneNorm", (FalconTransformerContainer, ),
                        {"__annotations__": {"qkv_w": GQAMegatronQKVParameter}})
        if getattr(cfg, "bias", False):
            raise NotImplementedError("biased Falcon checkpoints: use init_inference / build_hf_engine(model)")
        return FalconTransformerContainer if cfg.multi_query else FalconMHATransformerContainer


__all__ = [n for n in dir() if n.endswith(("Container", "Policy", "InferenceModel"))]
