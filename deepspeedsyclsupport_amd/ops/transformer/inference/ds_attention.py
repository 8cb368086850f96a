"""The two halves of the fused inference layer as modules of their own (reference
`ops/transformer/inference/ds_attention.py:17` `DeepSpeedSelfAttention` / `BloomSelfAttention`, `ds_mlp.py:14`
`DeepSpeedMLP`).

Both are views onto one `DeepSpeedTransformerInference` (the layer that owns the weights, the paged KV cache and the
position tables): `DeepSpeedSelfAttention` runs input norm -> QKV GEMM -> RoPE + cache append -> attention -> output
GEMM, `DeepSpeedMLP` runs residual add -> norm -> MLP -> residual add, through the same HIP kernels as the whole
layer. Constructed from a config they create their host layer; `from_layer` wraps an existing one.
"""
import torch
import torch.nn as nn

from .config import DeepSpeedInferenceConfig
from .layer import DeepSpeedTransformerInference


class DeepSpeedSelfAttention(nn.Module):
    num_layers = 0

    def __init__(self, config: DeepSpeedInferenceConfig, mp_group=None, q_scales=None, q_groups=1, merge_count=1,
                 host: DeepSpeedTransformerInference = None):
        super().__init__()
        self.config = config
        self.host = host if host is not None else DeepSpeedTransformerInference(config, mp_group)
        DeepSpeedSelfAttention.num_layers += 1

    @classmethod
    def from_layer(cls, layer: DeepSpeedTransformerInference):
        return cls(layer.config, host=layer)

    # the reference's parameter names
    attn_qkvw = property(lambda self: self.host.layer.qkv_w)
    attn_qkvb = property(lambda self: self.host.layer.qkv_b)
    attn_ow = property(lambda self: self.host.layer.o_w)
    attn_ob = property(lambda self: self.host.layer.o_b)

    @torch.no_grad()
    def forward(self, input, input_mask=None, head_mask=None, layer_past=None, get_present=False,
                encoder_hidden_states=None, encoder_attention_mask=None, output_attentions=False, norm_w=None,
                norm_b=None, alibi=None):
        """-> (attention output [B, S, H] incl. the output bias, key, value, context placeholder, normed input).
        `norm_w` / `norm_b` default to the host layer's input norm."""
        H = self.host
        L = H.layer
        B, n, _ = input.shape
        start = 0 if layer_past is None else int(layer_past[0].shape[2])
        meta = H._meta(B, n, start, fresh=layer_past is None)
        x = input.to(H.config.dtype)
        inp_norm = L._norm(x, norm_w if norm_w is not None else L.ln1_w, norm_b if norm_b is not None else L.ln1_b)
        out = L._attention(inp_norm, meta, H.cache, H.rope, H.alibi)
        key, value = H._presents(B, start + n) if get_present else (None, None)
        return out.to(input.dtype), key, value, None, inp_norm


class BloomSelfAttention(DeepSpeedSelfAttention):
    """ALiBi attention: the host layer's spec (`bigscience_bloom=True`) carries the slopes."""


class DeepSpeedMLP(nn.Module):

    def __init__(self, config: DeepSpeedInferenceConfig, mp_group=None, q_scales=None, q_groups=1, merge_count=1,
                 mlp_extra_grouping=False, host: DeepSpeedTransformerInference = None):
        super().__init__()
        self.config = config
        self.host = host if host is not None else DeepSpeedTransformerInference(config, mp_group)

    @classmethod
    def from_layer(cls, layer: DeepSpeedTransformerInference):
        return cls(layer.config, host=layer)

    attn_nw = property(lambda self: self.host.layer.ln2_w)
    attn_nb = property(lambda self: self.host.layer.ln2_b)
    inter_w = property(lambda self: self.host.layer.fc1_w)
    inter_b = property(lambda self: self.host.layer.fc1_b)
    output_w = property(lambda self: self.host.layer.fc2_w)
    output_b = property(lambda self: self.host.layer.fc2_b)

    @torch.no_grad()
    def forward(self, input, residual, residual_norm=None, bias=None):
        """input: attention output; residual: the layer input. Returns residual + input (+ bias) + MLP(norm(...)),
        i.e. the layer output of a sequential (mlp_after_attn) block."""
        L = self.host.layer
        dt = self.host.config.dtype
        x = input.to(dt) if bias is None else input.to(dt) + bias.to(dt)
        normed, res = L._norm(x, L.ln2_w, L.ln2_b, residual.to(dt))
        return (L._mlp(normed) + res).to(input.dtype)
