"""Llama / Llama-2 decoder (the BASELINE flagship: Llama-2-7B ZeRO-3 training), MI355X-native layer.

Layer layout chosen for the hardware:
  * fused QKV projection ([Hq+2Hk]·D × H) and fused gate_up projection (2I × H): one large GEMM each instead of
    three/two (hipBLASLt reaches 1.3-1.6 PF on these shapes vs ~1.2 PF on the 4096² ones, `profiles/`);
  * residual add fused into RMSNorm (one HBM pass: `ds_hip_ops.rms_fwd` with residual);
  * RoPE fused with the QKV split + 0213 head-major transpose (`qkv_rope_fwd`);
  * SwiGLU as one fused kernel over the gate_up output;
  * LM loss as a fused softmax-CE kernel whose backward overwrites the logits in place.
Weights are random-init (no network); HF-format state dicts convert with `from_hf_state_dict`.
"""
import math
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn

from ..ops import reference
from ..ops.attention import attention
from ..ops.transformer import functional as DF


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: Optional[int] = None
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    tie_word_embeddings: bool = False
    initializer_range: float = 0.02
    hidden_act: str = "silu"
    attention_bias: bool = False

    def __post_init__(self):
        if self.num_key_value_heads is None:
            self.num_key_value_heads = self.num_attention_heads

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    def num_params(self, include_embedding=True):
        H, I, L, V = self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size
        D = self.head_dim
        per_layer = H * (self.num_attention_heads + 2 * self.num_key_value_heads) * D + H * H + 3 * H * I + 2 * H
        emb = V * H * (1 if self.tie_word_embeddings else 2)
        return L * per_layer + H + (emb if include_embedding else 0)

    def flops_per_token(self, seq_len):
        """Training FLOPs/token: 6·N_dense + 12·L·H·S (attention scores+context, fwd+bwd, causal not halved —
        the standard MFU convention)."""
        return 6 * self.num_params() + 12 * self.num_hidden_layers * self.hidden_size * seq_len


def _mk(base, kw):
    base.update(kw)
    return LlamaConfig(**base)


def llama2_7b_config(**kw):
    return _mk(dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32,
                    num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=4096), kw)


def llama2_13b_config(**kw):
    return _mk(dict(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40, num_attention_heads=40), kw)


def llama2_70b_config(**kw):
    return _mk(dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
                    num_key_value_heads=8), kw)


class RMSNorm(nn.Module):

    def __init__(self, hidden, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden))
        self.eps = eps

    def forward(self, x, residual=None):
        return DF.rms_norm(x, self.weight, self.eps, residual)


class RotaryTables(nn.Module):
    """fp32 cos/sin tables [max_pos, rot/2] built on the host (no device trig), kept as non-persistent buffers."""

    def __init__(self, rot_dim, max_pos, base):
        super().__init__()
        cos, sin = reference.rope_tables(max_pos, rot_dim, base)
        self.register_buffer("cos", cos, persistent=False)
        self.register_buffer("sin", sin, persistent=False)

    def ensure(self, n):
        if n > self.cos.shape[0]:
            cos, sin = reference.rope_tables(max(n, 2 * self.cos.shape[0]), self.cos.shape[1] * 2, 10000.0,
                                             device=self.cos.device)
            self.cos, self.sin = cos, sin


class LlamaAttention(nn.Module):

    def __init__(self, cfg: LlamaConfig, layer_idx=0):
        super().__init__()
        self.cfg = cfg
        self.layer_idx = layer_idx
        self.nh, self.nkv, self.hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        self.qkv_proj = nn.Linear(cfg.hidden_size, (self.nh + 2 * self.nkv) * self.hd, bias=cfg.attention_bias)
        self.o_proj = nn.Linear(self.nh * self.hd, cfg.hidden_size, bias=False)
        # optional sequence-parallel (Ulysses) wrapper installed by parallel.sequence
        self.seq_parallel = None

    def forward(self, x, rope: RotaryTables, position_ids=None, pos_offset=0):
        B, S, _ = x.shape
        qkv = self.qkv_proj(x).view(B, S, self.nh + 2 * self.nkv, self.hd)
        q, k, v = DF.qkv_rope_split(qkv, rope.cos, rope.sin, self.nh, self.nkv, position_ids=position_ids,
                                    pos_offset=pos_offset, token_major=self.seq_parallel is None)
        if self.seq_parallel is not None:
            o = self.seq_parallel(q, k, v)  # [B, Hq, S, D] (local sequence shard)
        else:
            o = attention(q, k, v, causal=True)
        o = o.transpose(1, 2).reshape(B, S, self.nh * self.hd)
        return self.o_proj(o)


class LlamaMLP(nn.Module):

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_up_proj = nn.Linear(cfg.hidden_size, 2 * cfg.intermediate_size, bias=False)
        self.down_proj = nn.Linear(cfg.intermediate_size, cfg.hidden_size, bias=False)
        self.act = cfg.hidden_act

    def forward(self, x):
        return self.down_proj(DF.gated_activation(self.gate_up_proj(x), self.act))


class LlamaDecoderLayer(nn.Module):

    def __init__(self, cfg: LlamaConfig, layer_idx=0):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg, layer_idx)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.mlp = LlamaMLP(cfg)

    def forward(self, hidden, residual, rope, position_ids=None, pos_offset=0):
        # pre-norm with the residual add fused into the norm kernel: returns (normed, new_residual)
        if residual is None:
            normed, residual = self.input_layernorm(hidden), hidden
        else:
            normed, residual = self.input_layernorm(hidden, residual)
        attn = self.self_attn(normed, rope, position_ids, pos_offset)
        normed, residual = self.post_attention_layernorm(attn, residual)
        return self.mlp(normed), residual


class LlamaModel(nn.Module):

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.rope = RotaryTables(cfg.head_dim, cfg.max_position_embeddings, cfg.rope_theta)
        self.gradient_checkpointing = False
        self._ckpt_fn = None

    def forward(self, input_ids, position_ids=None, pos_offset=0):
        self.rope.ensure(input_ids.shape[1] + pos_offset)
        h = self.embed_tokens(input_ids)
        residual = None
        for layer in self.layers:
            if self.gradient_checkpointing and self.training:
                ckpt = self._ckpt_fn or _default_checkpoint
                h, residual = ckpt(layer, h, residual, self.rope, position_ids, pos_offset)
            else:
                h, residual = layer(h, residual, self.rope, position_ids, pos_offset)
        return self.norm(h, residual)[0]


def _default_checkpoint(layer, h, residual, rope, position_ids, pos_offset):
    import torch.utils.checkpoint as cp
    if residual is None:
        residual = torch.zeros_like(h)
    return cp.checkpoint(layer, h, residual, rope, position_ids, pos_offset, use_reentrant=False)


class LlamaForCausalLM(nn.Module):

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        self.model = LlamaModel(cfg)
        self.lm_head = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False)
        if cfg.tie_word_embeddings:
            self.lm_head.weight = self.model.embed_tokens.weight
        self.apply(self._init_weights)

    def _init_weights(self, m):
        std = self.config.initializer_range
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=std)

    def gradient_checkpointing_enable(self, checkpoint_fn=None):
        self.model.gradient_checkpointing = True
        self.model._ckpt_fn = checkpoint_fn

    def forward(self, input_ids, labels=None, position_ids=None, pos_offset=0, shift_labels=True):
        h = self.model(input_ids, position_ids, pos_offset)
        if labels is None:
            return self.lm_head(h)
        if shift_labels:
            # predict token t+1 from position t; drop the last position (no target)
            h = h[:, :-1]
            labels = labels[:, 1:]
        logits = self.lm_head(h.reshape(-1, h.shape[-1]))
        return DF.cross_entropy(logits, labels.reshape(-1), inplace_backward=True)

    # ----------------------------------------------------------------------------- HF checkpoint interop
    @torch.no_grad()
    def from_hf_state_dict(self, sd):
        """Load a HuggingFace Llama state dict (separate q/k/v, gate/up) into the fused layout."""
        own = {}
        for k, v in sd.items():
            k2 = k
            own[k2] = v
        L = self.config.num_hidden_layers
        out = {}
        for k, v in own.items():
            if ".self_attn.q_proj." in k or ".self_attn.k_proj." in k or ".self_attn.v_proj." in k:
                continue
            if ".mlp.gate_proj." in k or ".mlp.up_proj." in k:
                continue
            out[k] = v
        for i in range(L):
            p = f"model.layers.{i}."
            out[p + "self_attn.qkv_proj.weight"] = torch.cat([
                own[p + "self_attn.q_proj.weight"], own[p + "self_attn.k_proj.weight"],
                own[p + "self_attn.v_proj.weight"]
            ])
            out[p + "mlp.gate_up_proj.weight"] = torch.cat([own[p + "mlp.gate_proj.weight"],
                                                            own[p + "mlp.up_proj.weight"]])
        return self.load_state_dict(out, strict=False)
