"""Per-rank position-bias builders for models whose attention bias is indexed by head (reference
`module_inject/auto_tp_model_utils.py`): once AutoTP has divided the heads over the ranks, the model's own ALiBi
helper must return only this rank's heads. Each function computes the full tensor the way the HF model does and keeps
the rank's head range."""
import math

import torch

from .. import comm as dist


def _alibi_slopes(num_heads, device):
    base = 2 ** math.floor(math.log2(num_heads))
    slopes = torch.pow(2 ** (-(2 ** -(math.log2(base) - 3))), torch.arange(1, base + 1, device=device,
                                                                            dtype=torch.float32))
    if base != num_heads:
        extra_base = 2 ** (-(2 ** -(math.log2(2 * base) - 3)))
        n = min(base, num_heads - base)
        slopes = torch.cat([slopes, torch.pow(extra_base, torch.arange(1, 1 + 2 * n, 2, device=device,
                                                                        dtype=torch.float32))])
    return slopes


_TP = {"group": None, "size": None, "rank": None}


def set_tp_group(group=None, size=None, rank=None):
    """The tensor-parallel group whose ranks share the heads (default: every rank of the job)."""
    _TP.update(group=group, size=size, rank=rank)


def _my_heads(num_heads):
    if _TP["size"] is not None:
        world, rank = _TP["size"], _TP["rank"]
    elif not dist.is_initialized() or dist.get_world_size() == 1:
        return 0, num_heads
    else:
        world, rank = dist.get_world_size(), dist.get_rank()
    if world == 1:
        return 0, num_heads
    per = num_heads // world
    return rank * per, (rank + 1) * per


def build_bloom_alibi_tensor(attention_mask, num_heads, dtype):
    """BLOOM: [batch * local_heads, 1, seq] = slope_h * (cumulative position of each unmasked key)."""
    batch, seq = attention_mask.shape
    slopes = _alibi_slopes(num_heads, attention_mask.device)
    pos = ((attention_mask.cumsum(dim=-1) - 1) * attention_mask)[:, None, :]
    alibi = (slopes[None, :, None] * pos).to(dtype)                         # [B, H, S]
    lo, hi = _my_heads(num_heads)
    return alibi[:, lo:hi].reshape(batch * (hi - lo), 1, seq)


def get_alibi_mask(self, tensor, seq_length_with_past):
    """Baichuan: the model's cached [H, S, S] causal-plus-ALiBi mask, this rank's heads only. Bound as a method of the
    HF model (it reads `self.n_head` and the cache attributes the model keeps)."""
    n_head = getattr(self, "n_head", None) or self.config.num_attention_heads
    slopes = _alibi_slopes(n_head, tensor.device)
    pos = torch.arange(seq_length_with_past, device=tensor.device, dtype=torch.float32)
    bias = slopes[:, None, None] * pos[None, None, :]
    causal = torch.full((seq_length_with_past, seq_length_with_past), float("-inf"), device=tensor.device).triu(1)
    mask = (bias + causal[None]).to(tensor.dtype)
    lo, hi = _my_heads(n_head)
    return mask[lo:hi]


def build_mpt_alibi_tensor(self, num_heads, sequence_length, alibi_bias_max=8, device=None):
    """MPT: [local_heads, 1, seq] with slopes 2^(-alibi_bias_max * h / H) over relative positions 1-S .. 0."""
    pos = torch.arange(1 - sequence_length, 1, dtype=torch.int32, device=device).view(1, 1, sequence_length)
    pow2 = 2 ** math.ceil(math.log2(num_heads))
    base = torch.arange(1, pow2 + 1, dtype=torch.float32, device=device) * (alibi_bias_max / pow2)
    slopes = 1.0 / torch.pow(2, base)
    if pow2 != num_heads:
        slopes = torch.cat([slopes[1::2], slopes[::2]])[:num_heads]
    alibi = (pos * slopes.view(num_heads, 1, 1))
    lo, hi = _my_heads(num_heads)
    return alibi[lo:hi]


def build_mpt_atten_bias_tensor(self, device, dtype, attention_mask=None, prefix_mask=None, sequence_id=None):
    """MPT attention bias for this rank's heads: the model's own builder, then the head slice."""
    attn_bias, attention_mask = self._attn_bias_orig(device=device, dtype=dtype, attention_mask=attention_mask,
                                                     prefix_mask=prefix_mask, sequence_id=sequence_id)
    if attn_bias is not None and attn_bias.dim() == 4:
        lo, hi = _my_heads(attn_bias.shape[1])
        attn_bias = attn_bias[:, lo:hi]
    return attn_bias, attention_mask
