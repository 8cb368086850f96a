"""Injection policies: how to read a client layer's weights (reference `module_inject/policy.py`).

A `TransformerPolicy` wraps ONE layer module of the client model and returns its tensors in the order the fused
inference layer takes them. Custom architectures plug into kernel injection by subclassing it and passing
`injection_policy={ClientLayerClass: PolicyClass}` to `init_inference`.
"""
from abc import ABC, abstractmethod

import torch

from ..utils.types import ActivationFuncType, NormType

transformer_param_names = (
    "attn_qkvw", "attn_qkvb", "attn_ow", "attn_ob", "inter_w", "inter_b", "output_w", "output_b", "attn_nw",
    "attn_nb", "norm_w", "norm_b")


class DSPolicy(ABC):
    _orig_layer_class = None

    def __init__(self):
        self.cuda_graph_supported = False

    @abstractmethod
    def attention(self):
        """(qkv weight, qkv bias, output weight, output bias): [out, in] weights, fused qkv rows ordered q | k | v."""
        raise NotImplementedError


class TransformerPolicy(DSPolicy):
    # a client whose weights should be replaced by a Hugging Face class sets this (reference: used to locate layers)
    hf_model_config = None

    def __init__(self, inference=True, linear_layer=True, scale_attention=True, megatron_v2=False,
                 use_mup=False, mlp_act_func_type=ActivationFuncType.GELU, pre_attn_norm=True, use_load_prefix=False,
                 split_qkv=True, norm_type=NormType.LayerNorm):
        super().__init__()
        self.cuda_graph_supported = False
        self.inference = inference
        self.linear_layer = linear_layer          # False: HF Conv1D ([in, out]) weights, transposed on read
        self.scale_attention = scale_attention
        self.is_megatron_v2 = megatron_v2
        self.use_mup = use_mup
        self.mlp_act_func_type = mlp_act_func_type
        self.pre_attn_norm = pre_attn_norm
        self.use_load_prefix = use_load_prefix
        self.split_qkv = split_qkv
        self.norm_type = norm_type
        # how the fused layer must treat positions (overridden by concrete policies)
        self.rotary_dim = -1
        self.rotate_half = False
        self.rotate_every_two = False
        self.rope_theta = 10000.0
        self.num_kv = -1
        self.bigscience_bloom = False
        self.mlp_after_attn = True
        self.window_size = 0
        self.return_tuple = False

    @abstractmethod
    def get_hidden_heads(self):
        """(hidden size, attention heads, norm epsilon, intermediate size)."""
        raise NotImplementedError

    @abstractmethod
    def mlp(self, enable_training=False):
        """(first weight, first bias, second weight, second bias); gated MLPs return [gate | up] stacked rows."""
        raise NotImplementedError

    @abstractmethod
    def layernorm(self):
        """(post-attention / MLP norm weight, its bias, input / attention norm weight, its bias)."""
        raise NotImplementedError


def transpose(data):
    """[in, out] -> contiguous [out, in] (HF Conv1D weights)."""
    with torch.no_grad():
        return data.t().contiguous()


def _fit(dst, src):
    return src.reshape(dst.shape).to(dst.dtype)


def maybe_copy(module, sd, weight_quantizer, mp_replace, dst_name, src_name, qkv=False, megatron_v2=False,
               split_qkv=False, heads=1):
    """Copy `sd[src_name]` into `module.<dst_name>` if the state dict has it (checkpoint-driven loading of an
    already-built fused layer). `weight_quantizer` / `mp_replace` may be None; when given they quantise / shard."""
    if src_name not in sd:
        return
    src, dst = sd[src_name], getattr(module, dst_name)
    if mp_replace is not None:
        src = mp_replace.strided_copy(dst, src, num_splits=3) if (qkv and split_qkv) else mp_replace.copy(dst, src)
    if weight_quantizer is not None and src.dim() == 2:
        src = weight_quantizer.quantize(src)
    with torch.no_grad():
        dst.copy_(_fit(dst, src))


def maybe_copy_qkv(module, sd, weight_quantizer, mp_replace, dst_name, src_names, split_qkv=False):
    """Fuse separate q / k / v tensors of the state dict into `module.<dst_name>`."""
    if src_names[0] not in sd:
        return
    fused = torch.cat([sd[n] for n in src_names], dim=0)
    maybe_copy(module, {dst_name: fused}, weight_quantizer, mp_replace, dst_name, dst_name, qkv=True,
               split_qkv=split_qkv)


def maybe_copy_geglu(module, sd, weight_quantizer, mp_replace, dst_name, src_names):
    """Stack the gate and up projections of the state dict into `module.<dst_name>` as [gate | up]."""
    if src_names[0] not in sd:
        return
    fused = torch.cat([sd[src_names[0]], sd[src_names[1]]], dim=0)
    maybe_copy(module, {dst_name: fused}, weight_quantizer, mp_replace, dst_name, dst_name)


def pack_lora_weights(p):
    """[lora right, lora left, scaling] of a LoRA-wrapped linear, or [] (hybrid engine fuses them in place)."""
    return [p.lora_right_weight, p.lora_left_weight, p.lora_scaling] if hasattr(p, "lora_right_weight") else []


def maybe_get_lora(p):
    return pack_lora_weights(p)
