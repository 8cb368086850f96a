"""Standalone fused inference decoder layer (reference `ops/transformer/inference/ds_attention.py` +
`ds_mlp.py` + `model_implementations/transformers/ds_transformer.py:19` `DeepSpeedTransformerInference`, and
`moe_inference.py:186` `DeepSpeedMoEInference`).

The reference layer keeps a per-layer `layer_past` (K, V) and re-launches its CUDA attention over it. Here the layer
owns a paged KV cache (`inference/kv_cache.py` `BlockedKVCache`, one contiguous block run per batch row sized for
`max_out_tokens`), so a prompt is one flash prefill and each following token is one paged-decode step through the
same HIP kernels the kernel-injected engine uses. `layer_past` / the returned `presents` keep the reference's
contract: presents are the (K, V) tensors [B, Hk, L, D] viewed out of the cache, and passing them back continues the
sequence at position L."""
import math

import torch
import torch.nn as nn

from ....inference.model_implementations.transformer import BatchMeta, DSInferenceLayer, alibi_slopes
from ....inference.kv_cache import BlockedKVCache
from ... import reference
from .config import DeepSpeedInferenceConfig, DeepSpeedMoEInferenceConfig


class DeepSpeedTransformerInference(nn.Module):
    layer_id = 0

    def __init__(self, config: DeepSpeedInferenceConfig, mp_group=None, quantize_scales=None, quantize_groups=1,
                 merge_count=1, mlp_extra_grouping=False, device=None):
        super().__init__()
        self.config = config
        self.config.layer_id = DeepSpeedTransformerInference.layer_id
        DeepSpeedTransformerInference.layer_id += 1
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.spec = config.to_spec()
        tp = config.mp_size if mp_group is not None else 1
        self.layer = DSInferenceLayer(self.spec, 0, mp_group, tp, config.dtype, self.device)
        for p in self.layer.parameters():  # projections start random (load_weights overwrites); norms stay 1 / 0
            if p.dim() >= 2:
                nn.init.normal_(p, std=0.02)
        self.block_size = 64
        self.per_seq = -(-config.max_out_tokens // self.block_size)
        self.cache = None
        if self.spec.pos in ("rope", "rope_gptj"):
            cos, sin = reference.rope_tables(max(config.max_out_tokens, 2048), self.spec.rotary_dim,
                                             self.spec.rope_theta, device=self.device)
            self.rope = (cos, sin)
        else:
            self.rope = (None, None)
        if self.spec.pos == "alibi":
            hq = self.layer.hq
            rank = torch.distributed.get_rank(mp_group) if mp_group is not None else 0
            self.alibi = alibi_slopes(self.spec.num_heads)[rank * hq:(rank + 1) * hq].contiguous().to(self.device)
        else:
            self.alibi = None
        if config.scale_attn_by_inverse_layer_idx:
            self.spec.attn_scale = 1.0 / (math.sqrt(self.spec.head_dim) * (config.layer_id + 1))

    # ------------------------------------------------------------------------------------------ weights
    def load_weights(self, attn_qkvw, attn_ow, inter_w, output_w, attn_nw=None, norm_w=None, attn_qkvb=None,
                     attn_ob=None, inter_b=None, output_b=None, attn_nb=None, norm_b=None):
        """Copy a layer's tensors in ([out, in] weights, as nn.Linear stores them)."""
        L = self.layer
        with torch.no_grad():
            for dst, src in ((L.qkv_w, attn_qkvw), (L.o_w, attn_ow), (L.fc1_w, inter_w), (L.fc2_w, output_w),
                             (L.ln1_w, attn_nw), (L.ln2_w, norm_w), (L.qkv_b, attn_qkvb), (L.o_b, attn_ob),
                             (L.fc1_b, inter_b), (L.fc2_b, output_b), (L.ln1_b, attn_nb), (L.ln2_b, norm_b)):
                if dst is not None and src is not None:
                    dst.copy_(src.reshape(dst.shape))

    # ------------------------------------------------------------------------------------------ forward
    def _ensure_cache(self, batch):
        need = batch * self.per_seq
        if self.cache is None or self.cache.num_blocks < need:
            self.cache = BlockedKVCache(1, need, self.layer.hk, self.block_size, self.spec.head_dim,
                                        self.config.dtype, self.device)

    def _presents(self, B, L):
        k, v = self.cache.k[0], self.cache.v[0]
        nblk = -(-L // self.block_size)

        def view(c):
            c = c[:B * self.per_seq].view(B, self.per_seq, c.shape[1], self.block_size, c.shape[3])[:, :nblk]
            return c.permute(0, 2, 1, 3, 4).reshape(B, c.shape[2], nblk * self.block_size, c.shape[4])[:, :, :L]

        return view(k), view(v)

    def _meta(self, B, n, start, fresh):
        """Batch metadata of a step that appends `n` tokens at position `start` to each of `B` sequences."""
        if start + n > self.per_seq * self.block_size:
            raise ValueError(f"sequence length {start + n} exceeds max_out_tokens={self.config.max_out_tokens}")
        if fresh:
            self._ensure_cache(B)
        dev = self.device
        tables = torch.arange(B * self.per_seq, dtype=torch.int32, device=dev).view(B, self.per_seq)
        st = torch.full((B, ), start, dtype=torch.int32, device=dev)
        pos = (st[:, None] + torch.arange(n, dtype=torch.int32, device=dev)[None, :]).reshape(-1).contiguous()
        return BatchMeta(block_tables=tables, start_pos=st, seq_lens=st + n, pos_ids=pos, n_new=n,
                         max_len=self.per_seq * self.block_size, prefill_from_zero=start == 0)

    @torch.no_grad()
    def forward(self, input=None, input_mask=None, attention_mask=None, attn_mask=None, head_mask=None,
                layer_past=None, get_key_value=False, get_present=False, encoder_output=None, enc_dec_attn_mask=None,
                x=None, encoder_hidden_states=None, encoder_attention_mask=None, use_cache=False, alibi=None,
                output_attentions=False, layer_head_mask=None, past_key_value=None, **kwargs):
        h = x if x is not None else input
        if h is None:
            raise ValueError("DeepSpeedTransformerInference.forward needs `input` (or `x`)")
        mask = input_mask if input_mask is not None else (attention_mask if attention_mask is not None else attn_mask)
        if mask is not None and mask.dtype == torch.bool and not bool(mask.all()):
            raise ValueError("padding masks are not supported by the standalone layer: run padded batches through "
                             "`init_inference` (the engine unpads into a ragged batch)")
        past = layer_past if layer_past is not None else past_key_value
        B, n, _ = h.shape
        start = 0 if past is None else int(past[0].shape[2])
        meta = self._meta(B, n, start, fresh=past is None)
        inp = h.to(self.config.dtype)
        out, residual = self.layer(inp, None, meta, self.cache, self.rope, self.alibi)
        out = (out + residual).to(h.dtype)
        if get_present or use_cache or get_key_value:
            presents = self._presents(B, start + n)
            return (out, presents) if self.config.return_tuple or get_key_value else out
        return (out, ) if self.config.return_tuple else out


class DeepSpeedMoEInference(DeepSpeedTransformerInference):
    """Decoder layer whose MLP is top-k routed experts (grouped MFMA GEMM pair, `ops/moe_ops.py` `moe_block`)."""

    def __init__(self, config: DeepSpeedMoEInferenceConfig, mp_group=None, ep_group=None, expert_mp_group=None,
                 quantize_scales=None, quantize_groups=1, merge_count=1, mlp_extra_grouping=False, device=None):
        super().__init__(config, mp_group, quantize_scales, quantize_groups, merge_count, mlp_extra_grouping, device)
        self.ep_group = ep_group
        self.expert_mp_group = expert_mp_group
