"""Block-sparse self-attention (reference `ops/sparse_attention/sparse_self_attention.py`,
`bert_sparse_self_attention.py`, `sparse_attention_utils.py`).

16-bit device inputs run the block-sparse gfx950 flash kernels (`block_sparse.py`: only the key tiles the layout
touches are visited); key-padding masks, attention masks ('add' or 'mul' mode) and relative position embeddings are
applied inside those kernels, as the reference's sparse softmax does. Host / fp32 inputs take a dense reference
path: the block layout is expanded into a token-level additive mask and attention runs through SDPA. Layouts and
API are the reference's.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .sparsity_config import FixedSparsityConfig, SparsityConfig


class SparseSelfAttention(nn.Module):

    def __init__(self, sparsity_config: SparsityConfig = None, key_padding_mask_mode="add", attn_mask_mode="mul",
                 max_seq_length=2048):
        super().__init__()
        self.sparsity_config = sparsity_config or FixedSparsityConfig(num_heads=4)
        self.key_padding_mask_mode = key_padding_mask_mode
        self.attn_mask_mode = attn_mask_mode
        self.max_seq_length = max_seq_length
        self._masks = {}

    def get_layout(self, L):
        lay = self._layouts.get(L) if hasattr(self, "_layouts") else None
        if lay is None:
            if not hasattr(self, "_layouts"):
                self._layouts = {}
            lay = self._layouts[L] = self.sparsity_config.make_layout(L)
        return lay

    def _block_mask(self, L, device):
        key = (L, str(device))
        if key not in self._masks:
            layout = self.get_layout(L).bool()
            b = self.sparsity_config.block
            tok = layout.repeat_interleave(b, 1).repeat_interleave(b, 2)  # [H, L, L]
            self._masks[key] = torch.zeros(tok.shape, dtype=torch.float32, device=device).masked_fill_(
                ~tok.to(device), float("-inf"))
        return self._masks[key]

    @staticmethod
    def _as_additive(mask, mode, dtype):
        m = mask.to(torch.float32)
        if mode == "mul":  # 1 keep / 0 drop
            return torch.where(m > 0, 0.0, float("-inf"))
        return m

    def forward(self, query, key, value, rpe=None, key_padding_mask=None, attn_mask=None):
        B, H, L, D = query.shape
        if query.dtype not in (torch.float16, torch.bfloat16, torch.float32):
            raise TypeError("sparse attention supports fp16/bf16/fp32")
        from . import block_sparse
        blk = self.sparsity_config.block
        if block_sparse.native_ok(query, key, value, blk):
            # masks and relative position embeddings are applied inside the gfx950 kernels
            return block_sparse.block_sparse_attention(
                query, key, value, self.get_layout(L), blk, rpe=rpe, key_padding_mask=key_padding_mask,
                attn_mask=attn_mask, key_padding_mask_mode=self.key_padding_mask_mode,
                attn_mask_mode=self.attn_mask_mode)
        # host tensors / fp32: dense reference path
        bias = self._block_mask(L, query.device)[None]              # [1, H, L, L]
        if rpe is not None:
            bias = bias + rpe.float().view(-1, H, L, L) if rpe.dim() == 4 else bias + rpe.float()
        if key_padding_mask is not None:                             # [B, L]
            bias = bias + self._as_additive(key_padding_mask, self.key_padding_mask_mode,
                                            query.dtype).view(B, 1, 1, L)
        if attn_mask is not None:                                    # [L, L]
            bias = bias + self._as_additive(attn_mask, self.attn_mask_mode, query.dtype).view(1, 1, L, L)
        return F.scaled_dot_product_attention(query, key, value, attn_mask=bias.to(query.dtype))


class BertSparseSelfAttention(nn.Module):
    """Drop-in replacement for a BERT self-attention block using block-sparse attention."""

    def __init__(self, config, sparsity_config=None):
        super().__init__()
        if config.hidden_size % config.num_attention_heads:
            raise ValueError("hidden size must be a multiple of the number of heads")
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = config.hidden_size // config.num_attention_heads
        self.all_head_size = config.hidden_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        self.sparse_self_attention = SparseSelfAttention(
            sparsity_config or FixedSparsityConfig(num_heads=config.num_attention_heads))

    def _split(self, x):
        B, L, _ = x.shape
        return x.view(B, L, self.num_attention_heads, self.attention_head_size).transpose(1, 2)

    def forward(self, hidden_states, attention_mask=None):
        q, k, v = self._split(self.query(hidden_states)), self._split(self.key(hidden_states)), \
            self._split(self.value(hidden_states))
        ctx = self.sparse_self_attention(q, k, v, key_padding_mask=attention_mask)
        B, H, L, D = ctx.shape
        return ctx.transpose(1, 2).reshape(B, L, H * D)


class SparseAttentionUtils:

    @staticmethod
    def pad_to_block_size(block_size, input_ids, attention_mask, token_type_ids, position_ids, inputs_embeds,
                          pad_token_id, model_embeddings=None):
        L = (input_ids if input_ids is not None else inputs_embeds).shape[1]
        pad = (block_size - L % block_size) % block_size
        if pad:
            if input_ids is not None:
                input_ids = F.pad(input_ids, (0, pad), value=pad_token_id)
            if inputs_embeds is not None:
                fill = model_embeddings(torch.full((inputs_embeds.shape[0], pad), pad_token_id,
                                                   device=inputs_embeds.device)) if model_embeddings else \
                    inputs_embeds.new_zeros(inputs_embeds.shape[0], pad, inputs_embeds.shape[2])
                inputs_embeds = torch.cat([inputs_embeds, fill], 1)
            if attention_mask is not None:
                attention_mask = F.pad(attention_mask, (0, pad), value=0)
            if token_type_ids is not None:
                token_type_ids = F.pad(token_type_ids, (0, pad), value=0)
            if position_ids is not None:
                position_ids = F.pad(position_ids, (0, pad), value=pad_token_id)
        return pad, input_ids, attention_mask, token_type_ids, position_ids, inputs_embeds

    @staticmethod
    def unpad_sequence_output(pad_len, sequence_output):
        return sequence_output[:, :-pad_len] if pad_len > 0 else sequence_output

    @staticmethod
    def extend_position_embedding(model, max_position):
        """Tile a learned position embedding table to `max_position` rows."""
        emb = model.embeddings.position_embeddings if hasattr(model, "embeddings") else model
        old = emb.weight.data
        reps = -(-max_position // old.shape[0])
        new = nn.Embedding(max_position, old.shape[1]).to(old.device, old.dtype)
        new.weight.data.copy_(old.repeat(reps, 1)[:max_position])
        if hasattr(model, "embeddings"):
            model.embeddings.position_embeddings = new
        return model
