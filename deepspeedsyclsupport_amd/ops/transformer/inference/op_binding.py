"""Callable op objects of the v1 inference layer (reference `ops/transformer/inference/op_binding/*.py`: each wraps
one `transformer_inference` extension function chosen by dtype). Here each is a small composition of the gfx950
kernels behind `ops/transformer/functional.py` and the library GEMM; weights are [out, in] as nn.Linear stores them
unless `transposed_mode` is set on the config."""
import math

import torch
import torch.nn.functional as F

from ....utils.types import ActivationFuncType, NormType
from .. import functional as DF

__path__ = []  # lets the reference's per-op sub-paths resolve through `_import_paths`


class BaseOp(torch.nn.Module):
    inference_module = None

    def __init__(self, config):
        super().__init__()
        self.config = config

    def _w(self, weight):
        return weight.t() if getattr(self.config, "transposed_mode", False) else weight

    def _norm(self, x, gamma, beta):
        if self.config.norm_type == NormType.RMSNorm:
            return DF.rms_norm(x, gamma, self.config.layer_norm_eps)
        return DF.layer_norm(x, gamma, beta, self.config.layer_norm_eps)


class QKVGemmOp(BaseOp):
    """(norm(input) . W^T + b, norm(input))."""

    def forward(self, input, weight, q_scale=None, bias=None, gamma=None, beta=None):
        normed = self._norm(input, gamma, beta) if gamma is not None else input
        return F.linear(normed, self._w(weight), bias), normed


class LinearOp(BaseOp):

    def forward(self, input, weight, bias=None, add_bias=True, do_flash_attn=False, num_heads=1, external_cache=None,
                num_layers=1):
        return F.linear(input, self._w(weight), bias if add_bias else None)


class VectorMatMulOp(BaseOp):

    def forward(self, input, weight, async_op=False, q_scale=None, q_int8=False, transpose=False):
        return F.linear(input, weight.t() if transpose else self._w(weight))


class GELUGemmOp(BaseOp):
    """act(input . W1^T + b) . W2^T."""

    def forward(self, input, weight, bias, weight_out, async_op=False):
        return F.linear(DF.bias_activation(F.linear(input, self._w(weight)), bias, "gelu"), self._w(weight_out))


class MLPGemmOp(BaseOp):
    """residual_add = input + residual (+ input_bias); out = act(norm(residual_add) . W1^T + b1) . W2^T.
    Returns (out, residual_add)."""

    def forward(self, input, residual, weight_interm, weight_out, input_bias=None, bias=None, gamma=None, beta=None):
        x = input if input_bias is None else input + input_bias
        if self.config.norm_type == NormType.RMSNorm:
            normed, res = DF.rms_norm(x, gamma, self.config.layer_norm_eps, residual)
        else:
            normed, res = DF.layer_norm(x, gamma, beta, self.config.layer_norm_eps, residual)
        h = F.linear(normed, self._w(weight_interm))
        act = self.config.mlp_act_func_type
        if act in (ActivationFuncType.GATED_GELU, ActivationFuncType.GATED_SILU):
            h = DF.gated_activation(h if bias is None else h + bias,
                                    "gelu" if act == ActivationFuncType.GATED_GELU else "silu")
        else:
            h = DF.bias_activation(h, bias, "relu" if act == ActivationFuncType.ReLU else "gelu")
        return F.linear(h, self._w(weight_out)), res


class ResidualAddOp(BaseOp):
    """hidden_state + residual (+ biases), with the GPT-J / NeoX parallel form when `mlp_after_attn` is False:
    (residual + attention_output + attention_bias + hidden_state + final_bias), the tensor-parallel shares of the
    biases divided by `mp_size`."""

    def forward(self, hidden_state, residual, add_bias=True, attention_output=None, attention_bias=None,
                final_bias=None, residual_add=None):
        mp = max(getattr(self.config, "mp_size", 1), 1)
        if getattr(self.config, "mlp_after_attn", True):
            out = hidden_state + (residual_add if residual_add is not None else residual)
            if add_bias and final_bias is not None:
                out = out + final_bias
            return out
        out = hidden_state + residual
        if attention_output is not None:
            out = out + attention_output
        if add_bias:
            for b in (attention_bias, final_bias):
                if b is not None:
                    out = out + b / mp
        return out


class SoftmaxOp(BaseOp):
    """Masked, optionally ALiBi-biased and triangular softmax over attention scores [B, H, S, L]."""

    def forward(self, attn_scores, attn_mask=None, alibi=None, triangular=False, recompute=False,
                local_attention=False, window_size=256, async_op=False, layer_scale=1.0, head_offset=0):
        s = attn_scores.float() * layer_scale
        if alibi is not None:
            a = alibi.float()
            s = s + a.reshape(s.shape[0], -1, *a.shape[-2:])[:, head_offset:head_offset + s.shape[1]]
        if attn_mask is not None:
            s = s + attn_mask.float()
        S, Lk = s.shape[-2:]
        if triangular:
            q = torch.arange(Lk - S, Lk, device=s.device)[:, None]
            k = torch.arange(Lk, device=s.device)[None, :]
            bad = k > q
            if local_attention:
                bad = bad | (k <= q - window_size)
            s = s.masked_fill(bad, float("-inf"))
        return torch.softmax(s, dim=-1).to(attn_scores.dtype)


class SoftmaxContextOp(BaseOp):
    """Fused-QKV [B, S, (Hq + 2 Hkv) * D] -> causal attention context [B, S, Hq * D], plus this call's key and value
    [B, Hkv, S, D] (the standalone op keeps no cache: `DeepSpeedSelfAttention` is the cached path)."""

    def forward(self, query_key_value, attn_mask=None, heads=1, num_kv=-1, norm_factor=None, no_masking=False,
                layer_id=0, num_layers=1, alibi=None):
        B, S, W = query_key_value.shape
        hk = heads if num_kv is None or num_kv <= 0 else num_kv
        D = W // (heads + 2 * hk)
        q, k, v = query_key_value.view(B, S, heads + 2 * hk, D).split([heads, hk, hk], dim=2)
        q, k, v = (t.transpose(1, 2) for t in (q, k, v))
        rep = heads // hk
        kk, vv = (k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)) if rep > 1 else (k, v)
        scale = norm_factor * norm_factor if norm_factor is not None else 1.0 / math.sqrt(D)
        bias = None
        if alibi is not None:
            bias = alibi.float().reshape(B, heads, -1, S)[:, :, -1:, :].to(q.dtype)
        if attn_mask is not None:
            bias = attn_mask.to(q.dtype) if bias is None else bias + attn_mask.to(q.dtype)
        if bias is None:
            ctx = F.scaled_dot_product_attention(q, kk, vv, is_causal=not no_masking, scale=scale)
        else:
            if not no_masking:
                tri = torch.full((S, S), float("-inf"), device=q.device, dtype=q.dtype).triu(1)
                bias = bias + tri
            ctx = F.scaled_dot_product_attention(q, kk, vv, attn_mask=bias, scale=scale)
        return ctx.transpose(1, 2).reshape(B, S, heads * D), k, v
