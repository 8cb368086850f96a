"""Fused BERT-style training layer (reference `ops/transformer/transformer.py:21-420` DeepSpeedTransformerLayer /
DeepSpeedTransformerConfig and `csrc/transformer/ds_transformer_cuda.cpp:154-300`).

Same parameters (attn_qkvw/b, attn_ow/b, attn_nw/b, inter_w/b, output_w/b, norm_w/b) and pre-/post-LN semantics:
  pre-LN : x1 = LN_a(x);  r = x + drop(Attn(x1));  out = r + drop(FF(LN_n(r)))
  post-LN: r = LN_a(x + drop(Attn(x)));  out = LN_n(r + drop(FF(r)))
The MI355X pipeline: hipBLASLt GEMMs for QKV / O / FF1 / FF2, the fused small-head attention kernel
(`csrc/attn/flash_small.hip`: per-key additive BERT mask and attention-probability dropout in-kernel, reading Q/K/V
straight from the QKV GEMM output; SDPA for fp32 / host tensors / other head dims), gfx950 LayerNorm kernels with the residual add fused in, and the fused bias+GELU kernel; autograd
recomputation options map to activation checkpointing of the GELU output (gelu_checkpoint) and attention dropout
(attn_dropout_checkpoint).
"""
import json
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from . import functional as DF
from .. import flash_small as FS


def _per_key_mask(mask, B, S):
    """The additive BERT mask as [B, S] when it only varies per key ([B, S], [B, 1, 1, S] or [B, 1, S] forms)."""
    if mask is None:
        return None
    if mask.dim() == 2 and tuple(mask.shape) == (B, S):
        return mask
    if mask.dim() == 4 and mask.shape[1] == 1 and mask.shape[2] == 1 and mask.shape[3] == S and mask.shape[0] in (1, B):
        return mask[:, 0, 0, :].expand(B, S)
    if mask.dim() == 3 and mask.shape[1] == 1 and mask.shape[2] == S and mask.shape[0] in (1, B):
        return mask[:, 0, :].expand(B, S)
    return None


class TransformerConfig:

    def __init__(self, batch_size, hidden_size, intermediate_size, heads, attn_dropout_ratio, hidden_dropout_ratio,
                 num_hidden_layers, initializer_range):
        self.layer_id = -1
        self.batch_size = batch_size
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size
        self.heads = heads
        self.attn_dropout_ratio = attn_dropout_ratio
        self.hidden_dropout_ratio = hidden_dropout_ratio
        self.num_hidden_layers = num_hidden_layers
        self.initializer_range = initializer_range


class DeepSpeedTransformerConfig(TransformerConfig):

    def __init__(self, batch_size=-1, hidden_size=-1, intermediate_size=-1, heads=-1, attn_dropout_ratio=-1,
                 hidden_dropout_ratio=-1, num_hidden_layers=-1, initializer_range=-1, layer_norm_eps=1e-12,
                 local_rank=-1, seed=-1, fp16=False, pre_layer_norm=True, normalize_invertible=False,
                 gelu_checkpoint=False, adjust_init_range=True, attn_dropout_checkpoint=False, stochastic_mode=False,
                 return_tuple=False, training=True):
        super().__init__(batch_size, hidden_size,
                         intermediate_size if intermediate_size > 0 else 4 * hidden_size, heads,
                         attn_dropout_ratio, hidden_dropout_ratio, num_hidden_layers, initializer_range)
        self.fp16 = fp16
        self.pre_layer_norm = pre_layer_norm
        self.local_rank = local_rank
        self.seed = seed
        self.normalize_invertible = normalize_invertible
        self.gelu_checkpoint = gelu_checkpoint
        self.adjust_init_range = adjust_init_range
        self.test_gemm = False
        self.layer_norm_eps = layer_norm_eps
        self.training = training
        self.is_grad_enabled = True
        self.attn_dropout_checkpoint = attn_dropout_checkpoint
        self.stochastic_mode = stochastic_mode
        self.return_tuple = return_tuple

    @classmethod
    def from_dict(cls, json_object):
        cfg = cls()
        for k, v in json_object.items():
            cfg.__dict__[k] = v
        return cfg

    @classmethod
    def from_json_file(cls, json_file):
        with open(json_file, "r", encoding="utf-16") as f:
            return cls.from_dict(json.loads(f.read()))


class DeepSpeedTransformerLayer(nn.Module):
    layer_id = 0

    def __init__(self, config, initial_weights=None, initial_biases=None):
        super().__init__()
        self.config = config
        self.config.layer_id = DeepSpeedTransformerLayer.layer_id
        DeepSpeedTransformerLayer.layer_id += 1
        H, I = config.hidden_size, config.intermediate_size
        if initial_weights is None:
            self.attn_qkvw = nn.Parameter(torch.empty(3 * H, H))
            self.attn_qkvb = nn.Parameter(torch.empty(3 * H))
            self.attn_ow = nn.Parameter(torch.empty(H, H))
            self.attn_ob = nn.Parameter(torch.empty(H))
            self.attn_nw = nn.Parameter(torch.empty(H))
            self.attn_nb = nn.Parameter(torch.empty(H))
            self.inter_w = nn.Parameter(torch.empty(I, H))
            self.inter_b = nn.Parameter(torch.empty(I))
            self.output_w = nn.Parameter(torch.empty(H, I))
            self.output_b = nn.Parameter(torch.empty(H))
            self.norm_w = nn.Parameter(torch.empty(H))
            self.norm_b = nn.Parameter(torch.empty(H))
            self.init_transformer_weights(config.adjust_init_range)
        else:
            # [q, k, v, o, attn_norm, inter, output, norm] weights / biases (reference order)
            self.attn_qkvw = nn.Parameter(torch.cat([w.data for w in initial_weights[:3]]))
            self.attn_qkvb = nn.Parameter(torch.cat([b.data for b in initial_biases[:3]]))
            self.attn_ow, self.attn_ob = nn.Parameter(initial_weights[3].data), nn.Parameter(initial_biases[3].data)
            self.attn_nw, self.attn_nb = nn.Parameter(initial_weights[4].data), nn.Parameter(initial_biases[4].data)
            self.inter_w, self.inter_b = nn.Parameter(initial_weights[5].data), nn.Parameter(initial_biases[5].data)
            self.output_w, self.output_b = nn.Parameter(initial_weights[6].data), nn.Parameter(initial_biases[6].data)
            self.norm_w, self.norm_b = nn.Parameter(initial_weights[7].data), nn.Parameter(initial_biases[7].data)

    def init_transformer_weights(self, adjust_init_range=False):
        std = self.config.initializer_range
        out_std = std / math.sqrt(2.0 * self.config.num_hidden_layers) if adjust_init_range else std
        with torch.no_grad():
            self.attn_qkvw.normal_(0.0, std)
            self.attn_qkvb.zero_()
            self.attn_ow.normal_(0.0, out_std)
            self.attn_ob.zero_()
            self.attn_nw.fill_(1.0)
            self.attn_nb.zero_()
            self.inter_w.normal_(0.0, std)
            self.inter_b.zero_()
            self.output_w.normal_(0.0, out_std)
            self.output_b.zero_()
            self.norm_w.fill_(1.0)
            self.norm_b.zero_()

    def _ln(self, x, w, b, residual=None):
        return DF.layer_norm(x, w, b, self.config.layer_norm_eps, residual)

    def _attention(self, x, mask):
        B, S, H = x.shape
        nh = self.config.heads
        qkv = F.linear(x, self.attn_qkvw, self.attn_qkvb).view(B, S, 3, nh, H // nh)
        p = self.config.attn_dropout_ratio if self.training else 0.0
        key_mask = _per_key_mask(mask, B, S)
        if FS.supported(qkv) and (mask is None or key_mask is not None):
            # fused kernel: [B, S, nh, D] views of the QKV GEMM output, per-key mask and attention dropout in-kernel
            q, k, v = qkv.unbind(2)
            b1 = key_mask.to(qkv.dtype) if key_mask is not None else None
            ctx = FS.flash_small(q, k, v, b1, dropout_p=p)
            return F.linear(ctx.view(B, S, H), self.attn_ow)
        q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
        if mask is not None:
            mask = mask.to(q.dtype)
            if mask.dim() == 2:
                mask = mask[:, None, None, :]
        ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=p)
        ctx = ctx.transpose(1, 2).reshape(B, S, H)
        return F.linear(ctx, self.attn_ow)  # output bias is fused into the dropout kernel

    def _ff(self, x):
        h = F.linear(x, self.inter_w)
        if self.config.gelu_checkpoint and self.training:
            h = checkpoint(lambda t: DF.bias_activation(t, self.inter_b, "gelu"), h, use_reentrant=False)
        else:
            h = DF.bias_activation(h, self.inter_b, "gelu")
        return F.linear(h, self.output_w)  # output bias is fused into the dropout kernel

    def forward(self, hidden_states, attention_mask=None, head_mask=None, layer_head_mask=None,
                encoder_hidden_states=None, encoder_attention_mask=None, past_key_value=None,
                output_attentions=False, grads=None):
        self.config.is_grad_enabled = torch.is_grad_enabled()
        self.config.training = self.training
        pd = self.config.hidden_dropout_ratio if self.training else 0.0
        x = hidden_states
        if self.config.pre_layer_norm:
            a = DF.dropout(self._attention(self._ln(x, self.attn_nw, self.attn_nb), attention_mask), pd,
                           self.training, bias=self.attn_ob)
            normed, r = self._ln(a, self.norm_w, self.norm_b, residual=x)   # fused residual add + LN
            out = DF.dropout(self._ff(normed), pd, self.training, bias=self.output_b, residual=r)
        else:
            a = DF.dropout(self._attention(x, attention_mask), pd, self.training, bias=self.attn_ob)
            r, _ = self._ln(a, self.attn_nw, self.attn_nb, residual=x)
            f = DF.dropout(self._ff(r), pd, self.training, bias=self.output_b)
            out, _ = self._ln(f, self.norm_w, self.norm_b, residual=r)
        if self.config.return_tuple:
            return (out, )
        return out
