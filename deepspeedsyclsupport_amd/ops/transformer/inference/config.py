"""Config of the op-level inference layer (reference `ops/transformer/inference/config.py:15`
`DeepSpeedInferenceConfig`). Same constructor keywords; `to_spec()` lowers it onto the `DSModelSpec` that drives the
fused MI355X layer, so every option maps to a concrete kernel choice (norm kind, activation code, RoPE layout,
ALiBi, sliding window, GQA)."""
import json

import torch

from ....utils.types import ActivationFuncType, GATED_ACTIVATION_TYPES, NormType

_ACT = {ActivationFuncType.GELU: "gelu", ActivationFuncType.ReLU: "relu", ActivationFuncType.GATED_GELU: "gelu",
        ActivationFuncType.GATED_SILU: "silu", ActivationFuncType.UNKNOWN: "gelu"}


class DeepSpeedInferenceConfig:

    def __init__(self, hidden_size=-1, intermediate_size=-1, heads=-1, num_hidden_layers=-1, layer_norm_eps=1e-12,
                 local_rank=-1, mp_size=1, dtype=torch.float16, pre_layer_norm=True, norm_type=NormType.LayerNorm,
                 stochastic_mode=False, scale_attention=True, triangular_masking=True, local_attention=False,
                 window_size=256, rotary_dim=-1, rotate_half=False, rotate_every_two=True, return_tuple=True,
                 mlp_after_attn=True, mlp_act_func_type=ActivationFuncType.GELU, training_mp_size=1,
                 bigscience_bloom=False, max_out_tokens=1024, min_out_tokens=1, scale_attn_by_inverse_layer_idx=False,
                 use_triton=False, triton_autotune=False, num_kv=-1, rope_theta=10000, set_empty_params=False,
                 transposed_mode=False, **unused):
        self.layer_id = -1
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size if intermediate_size > 0 else 4 * hidden_size
        self.heads = heads
        self.num_hidden_layers = num_hidden_layers
        self.layer_norm_eps = layer_norm_eps
        self.local_rank = local_rank
        self.mp_size = mp_size
        self.dtype = dtype
        self.pre_layer_norm = pre_layer_norm
        self.norm_type = NormType(norm_type)
        self.stochastic_mode = stochastic_mode
        self.scale_attention = scale_attention
        self.triangular_masking = triangular_masking
        self.local_attention = local_attention
        self.window_size = window_size
        self.rotary_dim = rotary_dim
        self.rotate_half = rotate_half
        self.rotate_every_two = rotate_every_two
        self.return_tuple = return_tuple
        self.mlp_after_attn = mlp_after_attn
        self.shared_parallel_norm = True
        self.mlp_act_func_type = ActivationFuncType(mlp_act_func_type)
        self.training_mp_size = training_mp_size
        self.bigscience_bloom = bigscience_bloom
        self.max_out_tokens = max_out_tokens
        self.min_out_tokens = min_out_tokens
        self.scale_attn_by_inverse_layer_idx = scale_attn_by_inverse_layer_idx
        self.num_kv = num_kv
        self.rope_theta = rope_theta
        if use_triton:
            raise ValueError("use_triton: there is no Triton path on MI355X; the layer runs hand-written HIP kernels")
        if not pre_layer_norm:
            raise ValueError("pre_layer_norm=False (post-LN) inference layers are not supported; the fused layer "
                             "is pre-norm")
        if not triangular_masking:
            raise ValueError("triangular_masking=False (bidirectional encoder) layers are served by "
                             "`DeepSpeedTransformerLayer` (ops/transformer/transformer.py), not the decoder layer")

    @classmethod
    def from_dict(cls, json_object):
        return cls(**json_object)

    @classmethod
    def from_json_file(cls, json_file):
        with open(json_file, "r", encoding="utf-8") as f:
            return cls.from_dict(json.load(f))

    def to_spec(self):
        from ....inference.model_implementations.transformer import DSModelSpec
        head_dim = self.hidden_size // self.heads
        if self.bigscience_bloom:
            pos, rot = "alibi", 0
        elif self.rotary_dim > 0:
            pos, rot = ("rope" if self.rotate_half else "rope_gptj"), self.rotary_dim
        else:
            pos, rot = "none", 0
        gated = self.mlp_act_func_type in GATED_ACTIVATION_TYPES
        return DSModelSpec(arch="ds_op_layer", vocab_size=1, hidden_size=self.hidden_size,
                           num_layers=max(self.num_hidden_layers, 1), num_heads=self.heads,
                           num_kv_heads=self.num_kv if self.num_kv > 0 else self.heads,
                           intermediate_size=self.intermediate_size, head_dim=head_dim,
                           norm="rms" if self.norm_type == NormType.RMSNorm else "ln", norm_eps=self.layer_norm_eps,
                           pos=pos, rope_theta=float(self.rope_theta), rotary_dim=rot,
                           act=_ACT[self.mlp_act_func_type], gated_mlp=gated,
                           qkv_bias=self.norm_type != NormType.RMSNorm, o_bias=self.norm_type != NormType.RMSNorm,
                           mlp_bias=self.norm_type != NormType.RMSNorm, max_positions=self.max_out_tokens,
                           sliding_window=self.window_size if self.local_attention else 0,
                           attn_scale=0.0 if self.scale_attention else 1.0,
                           # mlp_after_attn=False: attention and MLP both read the layer input and are summed with it
                           # (GPT-J: off ONE LayerNorm; GPT-NeoX: each off its own -> shared_parallel_norm False)
                           parallel_residual=not self.mlp_after_attn,
                           shared_parallel_norm=(not self.mlp_after_attn) and self.shared_parallel_norm)


class DeepSpeedMoEInferenceConfig(DeepSpeedInferenceConfig):
    """Reference `ops/transformer/inference/moe_inference.py:22`: adds the expert count / top-k of the MoE MLP."""

    def __init__(self, hidden_size=-1, intermediate_size=-1, heads=-1, num_hidden_layers=-1, layer_norm_eps=1e-12,
                 local_rank=-1, mp_size=1, fp16=False, bf16=False, q_int8=False, pre_layer_norm=True,
                 stochastic_mode=False, scale_attention=True, triangular_masking=True, local_attention=False,
                 window_size=256, return_tuple=True, moe_experts=1, global_experts=1, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, min_capacity=1, noisy_gate_policy=None, drop_tokens=True,
                 use_rts=False, mlp_type="standard", scale_attn_by_inverse_layer_idx=False, **kw):
        dtype = torch.bfloat16 if bf16 else (torch.float16 if fp16 else torch.float32)
        super().__init__(hidden_size, intermediate_size, heads, num_hidden_layers, layer_norm_eps, local_rank,
                         mp_size, dtype, pre_layer_norm, stochastic_mode=stochastic_mode,
                         scale_attention=scale_attention, triangular_masking=triangular_masking,
                         local_attention=local_attention, window_size=window_size, return_tuple=return_tuple,
                         scale_attn_by_inverse_layer_idx=scale_attn_by_inverse_layer_idx, **kw)
        self.moe_experts = moe_experts
        self.global_experts = global_experts
        self.k = k
        self.capacity_factor = capacity_factor
        self.eval_capacity_factor = eval_capacity_factor
        self.min_capacity = min_capacity
        self.noisy_gate_policy = noisy_gate_policy
        self.drop_tokens = drop_tokens
        self.use_rts = use_rts
        self.mlp_type = mlp_type
        self.q_int8 = q_int8

    def to_spec(self):
        spec = super().to_spec()
        spec.num_experts = max(int(self.moe_experts), 1)
        spec.moe_top_k = int(self.k)
        spec.moe_renormalize = self.k > 1
        return spec
