"""Kernel injection for encoders: BERT / RoBERTa / XLM-R / ELECTRA / CamemBERT layers, DistilBERT blocks and CLIP
(text + vision) encoder layers (reference `module_inject/containers/bert.py`, `containers/distil_bert.py`,
`containers/clip.py`, the policy-driven
`replace_transformer_layer` of `module_inject/replace_module.py:182` and the inference transformer it builds,
`model_implementations/transformers/ds_bert.py` over `ops/transformer/inference/ds_attention.py`).

Unlike decoders (converted whole into `DSInferenceModel` with a paged KV cache), an encoder has no cache and its
embeddings / pooler / heads stay the HF modules: each encoder layer is swapped IN PLACE for a `DSEncoderLayer`
that keeps the HF call contract (hidden_states, attention_mask, ...) -> hidden_states, so every task head
(MaskedLM, SequenceClassification, QA, ...) keeps working.

`DSEncoderLayer` (post-LN, the BERT family's layout):
  qkv    = x . Wqkv^T + b                 one GEMM over the concatenated q|k|v weights (bias in the GEMM epilogue)
  ctx    = attention(q, k, v, mask)       the small-head flash kernel (head dim 32 / 64) reading q/k/v as strided
                                          views of the fused projection, the padding mask as its per-key bias
                                          (other head dims: the library attention)
  x1     = LN(ctx . Wo^T + bo + x)        GEMM (+bias epilogue), then the fused residual-add + LayerNorm kernel
  h      = gelu(x1 . W1^T + b1)           GEMM, then the fused bias + GELU kernel
  out    = LN(h . W2^T + b2 + x1)         GEMM (+bias epilogue), fused residual-add + LayerNorm
CLIP layers are pre-LN (x1 = x + attn(LN1(x)); out = x1 + mlp(LN2(x1)), the second LayerNorm fused with the
residual add) with quick-GELU, and the text tower's causal mask arrives as `is_causal`.
Tensor parallelism shards q/k/v and W1 by output rows (heads / intermediate), Wo and W2 by input columns, with one
all-reduce after each row-parallel GEMM (bias added once, after the reduction).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist
from ..ops import flash_small as FS
from ..ops.transformer import functional as DF

_BERT_LIKE = ("BertLayer", "RobertaLayer", "XLMRobertaLayer", "ElectraLayer", "CamembertLayer", "RobertaPreLayerNormLayer")
_DISTIL = ("TransformerBlock", )
_CLIP = ("CLIPEncoderLayer", )
_ACTS = {"gelu": "gelu", "gelu_new": "gelu_tanh", "gelu_pytorch_tanh": "gelu_tanh", "relu": "relu", "silu": "silu"}


def _is_bert_layer(m):
    return type(m).__name__ in _BERT_LIKE and hasattr(m, "attention") and hasattr(m.attention, "self") \
        and hasattr(m.attention.self, "query") and not getattr(m, "is_decoder", False)


def _is_distil_block(m):
    return type(m).__name__ in _DISTIL and hasattr(m, "attention") and hasattr(m.attention, "q_lin") \
        and hasattr(m, "ffn")


def _is_clip_layer(m):
    return type(m).__name__ in _CLIP and hasattr(m, "self_attn") and hasattr(m.self_attn, "q_proj") \
        and hasattr(m, "layer_norm1") and hasattr(m, "mlp")


def supported(model):
    return any(_is_bert_layer(m) or _is_distil_block(m) or _is_clip_layer(m) for m in model.modules())


class DSEncoderLayer(nn.Module):

    def __init__(self, q, k, v, o, ln1, w1, w2, ln2, num_heads, act, tp_group=None, tp_size=1, tp_rank=0,
                 dtype=torch.bfloat16, device=None, pre_ln=False):
        super().__init__()
        self.pre_ln = pre_ln
        H = q.weight.shape[1]
        assert num_heads % tp_size == 0, "heads must divide the tensor-parallel size"
        self.nh = num_heads // tp_size
        self.hd = H // num_heads
        self.tp_group, self.tp = tp_group, tp_size
        self.act = _ACTS.get(act)            # None: no fused kernel for it (quick_gelu) -> torch epilogue
        self.act_name = act
        self.eps1, self.eps2 = ln1.eps, ln2.eps
        kw = dict(dtype=dtype, device=device)

        def rows(t, r=tp_rank):
            n = t.shape[0] // tp_size
            return t[r * n:(r + 1) * n]

        def cols(t, r=tp_rank):
            n = t.shape[1] // tp_size
            return t[:, r * n:(r + 1) * n]

        def p(t):
            return nn.Parameter(t.detach().to(**kw).contiguous(), requires_grad=False)

        self.qkv_w = p(torch.cat([rows(q.weight), rows(k.weight), rows(v.weight)], 0))
        self.qkv_b = p(torch.cat([rows(q.bias), rows(k.bias), rows(v.bias)], 0))
        self.o_w, self.o_b = p(cols(o.weight)), p(o.bias)
        self.ln1_w, self.ln1_b = p(ln1.weight), p(ln1.bias)
        self.w1, self.b1 = p(rows(w1.weight)), p(rows(w1.bias))
        self.w2, self.b2 = p(cols(w2.weight)), p(w2.bias)
        self.ln2_w, self.ln2_b = p(ln2.weight), p(ln2.bias)

    def _row_parallel(self, x, w, b):
        if self.tp == 1:
            return F.linear(x, w, b)
        y = F.linear(x, w)
        dist.all_reduce(y, group=self.tp_group)
        return y + b

    @staticmethod
    def _mask(mask, dtype):
        if mask is None:
            return None
        if mask.dim() == 2:  # [B, S] 1 = keep
            mask = mask[:, None, None, :].bool()
        if mask.dtype == torch.bool:
            return mask
        return mask.to(dtype)

    def _attn(self, x, attention_mask, is_causal):
        B, S, _ = x.shape
        qkv = F.linear(x, self.qkv_w, self.qkv_b).view(B, S, 3, self.nh, self.hd)
        causal = bool(is_causal and attention_mask is None)
        ctx = None
        if x.is_cuda and not torch.is_grad_enabled():
            raw = attention_mask  # as given: an expanded (stride-0) padding mask is recognised by its strides
            if raw is not None and raw.dim() == 2:
                raw = raw[:, None, None, :].bool()
            ctx = FS.attend(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], mask=raw, causal=causal)
        if ctx is None:
            mask = self._mask(attention_mask, qkv.dtype)
            q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
            ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, is_causal=causal).transpose(1, 2)
        return self._row_parallel(ctx.reshape(B, S, self.nh * self.hd), self.o_w, self.o_b)

    def _mlp(self, x):
        if self.act is not None:
            h = DF.bias_activation(F.linear(x, self.w1), self.b1, self.act)
        else:
            h = F.linear(x, self.w1, self.b1)
            h = h * torch.sigmoid(1.702 * h) if self.act_name == "quick_gelu" else F.gelu(h)
        return self._row_parallel(h, self.w2, self.b2)

    def forward(self, hidden_states, attention_mask=None, *args, **kwargs):
        x = hidden_states
        is_causal = kwargs.get("is_causal", False)
        if self.pre_ln:
            h = DF.layer_norm(x, self.ln1_w, self.ln1_b, self.eps1)
            a = self._attn(h, attention_mask, is_causal)
            h2, x1 = DF.layer_norm(a, self.ln2_w, self.ln2_b, self.eps2, residual=x)  # x1 = x + attn
            return x1 + self._mlp(h2)
        a = self._attn(x, attention_mask, is_causal)
        x1, _ = DF.layer_norm(a, self.ln1_w, self.ln1_b, self.eps1, residual=x)
        out, _ = DF.layer_norm(self._mlp(x1), self.ln2_w, self.ln2_b, self.eps2, residual=x1)
        return out


def _from_bert(m, cfg, **kw):
    a = m.attention
    return DSEncoderLayer(a.self.query, a.self.key, a.self.value, a.output.dense, a.output.LayerNorm,
                          m.intermediate.dense, m.output.dense, m.output.LayerNorm, cfg.num_attention_heads,
                          getattr(cfg, "hidden_act", "gelu"), **kw)


def _from_distil(m, cfg, **kw):
    a = m.attention
    return DSEncoderLayer(a.q_lin, a.k_lin, a.v_lin, a.out_lin, m.sa_layer_norm, m.ffn.lin1, m.ffn.lin2,
                          m.output_layer_norm, getattr(cfg, "n_heads", None) or cfg.num_attention_heads,
                          getattr(cfg, "activation", "gelu"), **kw)


def _from_clip(m, cfg, **kw):
    a = m.self_attn
    heads = getattr(a, "num_heads", None) or cfg.num_attention_heads
    act = getattr(getattr(a, "config", None), "hidden_act", None) or getattr(cfg, "hidden_act", "quick_gelu")
    return DSEncoderLayer(a.q_proj, a.k_proj, a.v_proj, a.out_proj, m.layer_norm1, m.mlp.fc1, m.mlp.fc2,
                          m.layer_norm2, heads, act, pre_ln=True, **kw)


def inject(model, tp_group=None, tp_size=1, tp_rank=0, dtype=torch.bfloat16, device=None):
    """Replace every encoder layer of `model` in place; the rest of the model is cast / moved to (dtype, device).
    Returns the number of layers replaced."""
    cfg = model.config
    kw = dict(tp_group=tp_group, tp_size=tp_size, tp_rank=tp_rank, dtype=dtype, device=device)
    n = 0
    for parent in list(model.modules()):
        for name, child in list(parent.named_children()):
            if _is_bert_layer(child):
                if getattr(child, "crossattention", None) is not None:
                    continue  # cross-attention decoder layers keep the HF implementation
                setattr(parent, name, _from_bert(child, cfg, **kw))
                n += 1
            elif _is_distil_block(child):
                setattr(parent, name, _from_distil(child, cfg, **kw))
                n += 1
            elif _is_clip_layer(child):
                setattr(parent, name, _from_clip(child, cfg, **kw))
                n += 1
    model.to(device=device, dtype=dtype)
    return n
