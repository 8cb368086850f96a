"""Ragged-batch kernel objects of inference v2 (reference `inference/v2/kernels/ragged_ops/{atom_builder,
blocked_flash,embed,linear_blocked_kv_rotary,logits_gather,moe_gather,moe_scatter,top_k_gating}`).

MI355X mapping. The reference splits attention into "atoms" built on the device and a blocked flash kernel that
walks them, with a separate kernel that rotates q / k and copies k / v into the blocked cache. Here:
  * the KV cache of a layer is two tensors `[blocks, kv_heads, block_size, head_dim]`; kernels take them as the pair
    `(k_cache, v_cache)` (a stacked `[2, blocks, ...]` tensor is accepted too);
  * `BlockedRotaryEmbeddings` / `BlockedTrainedRotaryEmbeddings` / `LinearBlockedKVCopy` are one fused epilogue
    (`csrc/attn/decode_attn.hip: qkv_rope_append`): rotate q and k in fp32, append k / v to the paged cache at each
    token's slot, return q — on the device for bf16, a torch fallback otherwise;
  * `AtomBuilder` produces the (sequence, 128-row query block) work list of the paged prefill kernel; the ragged
    wrapper already holds it (built on the host with the rest of the metadata, one upload);
  * `BlockedFlashAttn` runs `paged_decode` over the leading single-token sequences and `paged_prefill` over the
    prompt / chunk sequences (`csrc/attn/{decode_attn,paged_prefill}.hip`, head dims 64 / 80 / 96 / 128 / 256);
  * embedding / logits gathers and the MoE gating / scatter / gather are the row kernels of `csrc/moe/moe_kernels.hip`
    (`ops/moe_ops.py`), with torch fallbacks for host tensors.
Every object takes the `RaggedBatchWrapper` of the step and reads its device tables from `.meta`.
"""
import math
from typing import Optional, Tuple

import torch

from ....ops import moe_ops
from ....ops import reference as ref_ops
from ....ops.transformer import functional as DF
from ...model_implementations import transformer as T
from ..inference_utils import DtypeEnum
from .core_ops import _check_dtype
from .ds_kernel import DSKernelBase

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`

HEAD_SIZES = tuple(T.PAGED_HEAD_DIMS)


def _kv_pair(kv_cache):
    if isinstance(kv_cache, (tuple, list)):
        return kv_cache[0], kv_cache[1]
    if kv_cache.dim() == 5 and kv_cache.shape[0] == 2:
        return kv_cache[0], kv_cache[1]
    raise ValueError("kv_cache must be the pair (k_cache, v_cache) of [blocks, kv_heads, block_size, head_dim]")


def get_q_block_size(head_size: int) -> int:
    """Query rows one paged-prefill workgroup owns."""
    return 128


def get_kv_block_size(head_size: int) -> int:
    """Keys per inner step of the paged-prefill kernel."""
    return 64


class AtomBuilder(DSKernelBase):
    """Work list of the prefill kernel: rows (sequence index, query block) for every prompt / chunk sequence."""

    def __init__(self) -> None:
        pass

    def __call__(self, atoms: Optional[torch.Tensor], ragged_batch, q_block_size: int = 128,
                 kv_block_size: int = 64) -> Tuple[torch.Tensor, int]:
        if q_block_size != 128:
            raise ValueError("the paged prefill kernel owns 128 query rows per workgroup")
        work = ragged_batch.meta.work
        if atoms is not None and atoms.numel() >= work.numel():
            atoms.view(-1)[:work.numel()].copy_(work.view(-1))
        return work, work.shape[0]


class BlockedFlashAttn(DSKernelBase):
    """Causal attention of every token of the ragged batch over its sequence's paged KV (new tokens appended
    beforehand)."""
    supported_dtypes = [DtypeEnum.fp16, DtypeEnum.bf16, DtypeEnum.fp32]

    def __init__(self, head_size: int, dtype: DtypeEnum) -> None:
        self.dtype = _check_dtype(dtype, self.supported_dtypes)
        if head_size % 8 != 0:
            raise ValueError("Head size must be divisible by 8 (got {})".format(head_size))
        self.head_size = head_size

    def __call__(self, out: torch.Tensor, q: torch.Tensor, kv_cache, ragged_batch, softmax_scale: float = None,
                 alibi: Optional[torch.Tensor] = None, window: int = 0) -> torch.Tensor:
        """q [tokens, q_heads * head_size] (or [tokens, q_heads, head_size]) -> out, same shape."""
        kc, vc = _kv_pair(kv_cache)
        D = self.head_size
        q3 = q.reshape(q.shape[0], -1, D)
        scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
        o = T._ragged_attention(q3, kc, vc, ragged_batch.meta, scale, alibi, window)
        out.copy_(o.reshape(out.shape))
        return out


class _RotaryAppendBase(DSKernelBase):
    supported_dtypes = [DtypeEnum.fp16, DtypeEnum.bf16, DtypeEnum.fp32]
    supported_head_sizes = list(HEAD_SIZES)

    def _setup(self, head_size, n_q_heads, n_kv_heads, dtype):
        if head_size not in self.supported_head_sizes:
            raise ValueError(f"Unsupported head size: {head_size}, supported_head_sizes are "
                             f"{self.supported_head_sizes}")
        if n_q_heads % n_kv_heads != 0:
            raise ValueError(f"Unsupported q_ratio: {n_q_heads} query heads over {n_kv_heads} kv heads")
        self.dtype = _check_dtype(dtype, self.supported_dtypes)
        self.head_size, self.hq, self.hk = head_size, n_q_heads, n_kv_heads

    def _run(self, kv_cache, qkv, ragged_batch, cos, sin, rot, interleaved=False):
        kc, vc = _kv_pair(kv_cache)
        meta = ragged_batch.meta
        Tn, D = qkv.shape[0], self.head_size
        if qkv.is_cuda and qkv.dtype == torch.bfloat16 and kc.dtype == torch.bfloat16:
            from ....ops.native import hip_ops
            q = hip_ops().qkv_rope_append(qkv.contiguous(), cos if rot else None, sin if rot else None, meta.pos_ids,
                                          kc, vc, meta.block_tables, meta.start_pos, 1, self.hq, self.hk, rot,
                                          interleaved, False, meta.seq_ids, 0, None)[0]
        else:
            q, k, v = qkv.reshape(1, Tn, self.hq + 2 * self.hk, D).split([self.hq, self.hk, self.hk], dim=2)
            q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
            if rot:
                pos = meta.pos_ids.view(1, Tn)
                DF.apply_rotary_pos_emb(q, cos, sin, position_ids=pos, rotary_dim=rot, interleaved=interleaved)
                DF.apply_rotary_pos_emb(k, cos, sin, position_ids=pos, rotary_dim=rot, interleaved=interleaved)
            T._kv_append_ragged(k[0], v[0], kc, vc, meta)
            q = q[0]
        return q.reshape(Tn, self.hq * D)   # rotated queries (qkv itself is left as it was)


class BlockedRotaryEmbeddings(_RotaryAppendBase):
    """Rotate q / k with frequencies theta_base^(-2i / rotary_dim) and append k / v to the paged cache."""

    def __init__(self, head_size: int, n_q_heads: int, n_kv_heads: int, dtype: torch.dtype, rotary_dim: int,
                 theta_base: float, max_positions: int = 8192) -> None:
        self._setup(head_size, n_q_heads, n_kv_heads, dtype)
        if rotary_dim % 2 or rotary_dim > head_size:
            raise ValueError(f"rotary_dim {rotary_dim} must be even and at most the head size {head_size}")
        self.rotary_dim, self.theta_base, self.max_positions = rotary_dim, theta_base, max_positions
        self._tables = {}

    def _cos_sin(self, device, need):
        key = str(device)
        tab = self._tables.get(key)
        if tab is None or tab[0].shape[0] < need:
            n = max(self.max_positions, need)
            tab = self._tables[key] = ref_ops.rope_tables(n, self.rotary_dim, self.theta_base, device=device)
        return tab

    def __call__(self, kv_cache, qkv: torch.Tensor, ragged_batch) -> torch.Tensor:
        cos, sin = self._cos_sin(qkv.device, ragged_batch.meta.max_len + 1)
        return self._run(kv_cache, qkv, ragged_batch, cos, sin, self.rotary_dim)


class BlockedTrainedRotaryEmbeddings(_RotaryAppendBase):
    """As above with caller-provided inverse frequencies [max_seq_len, rotary_dim // 2] (angle per position)."""

    def __init__(self, head_size: int, n_q_heads: int, n_kv_heads: int, dtype: torch.dtype) -> None:
        self._setup(head_size, n_q_heads, n_kv_heads, dtype)

    def __call__(self, kv_cache, qkv: torch.Tensor, ragged_batch, inverse_freqs: torch.Tensor) -> torch.Tensor:
        ang = inverse_freqs.float()
        return self._run(kv_cache, qkv, ragged_batch, ang.cos(), ang.sin(), 2 * inverse_freqs.shape[-1])


class LinearBlockedKVCopy(_RotaryAppendBase):
    """Append k / v to the paged cache without rotation (learned / ALiBi position models)."""

    def __init__(self, head_size: int, n_q_heads: int, n_kv_heads: int, dtype: torch.dtype) -> None:
        self._setup(head_size, n_q_heads, n_kv_heads, dtype)

    def __call__(self, kv_cache, qkv: torch.Tensor, ragged_batch) -> torch.Tensor:
        return self._run(kv_cache, qkv, ragged_batch, None, None, 0)


class RaggedEmbeddingKernel(DSKernelBase):
    """embedded_tokens[t] = embedding_weight[token t] (+ position_embed_weight[position t + offset])."""
    supported_dtypes = [torch.float16, torch.bfloat16, torch.float32]
    supported_token_dtypes = [torch.int32, torch.int64]

    def __init__(self, embed_dtype: torch.dtype, token_dtype: torch.dtype, embed_dim: int) -> None:
        self.dtype = _check_dtype(embed_dtype, self.supported_dtypes, "embedding data type")
        if token_dtype not in self.supported_token_dtypes:
            raise ValueError(f"Unsupported token data type: {token_dtype}, supported_dtypes are "
                             f"{self.supported_token_dtypes}")
        self.embed_dim = embed_dim

    def __call__(self, embedded_tokens: torch.Tensor, ragged_wrapper, embedding_weight: torch.Tensor,
                 position_embed_weight: Optional[torch.Tensor] = None, position_embed_offset: int = 0) -> torch.Tensor:
        ids = ragged_wrapper.input_ids()
        pos = None
        if position_embed_weight is not None:
            pos = ragged_wrapper.meta.pos_ids.long() + position_embed_offset
        out = moe_ops.embed_gather(embedding_weight, ids, position_embed_weight, pos)
        embedded_tokens.copy_(out.view(embedded_tokens.shape))
        return embedded_tokens


class RaggedLogitsGather(DSKernelBase):
    """final_token_activations[s] = all_activations[last token row of sequence s] (kernel order)."""
    supported_dtypes = [torch.float16, torch.bfloat16, torch.float32]

    def __init__(self, model_dim: int, fp_dtype: torch.dtype):
        self.dtype = _check_dtype(fp_dtype, self.supported_dtypes)
        if model_dim % 8 != 0:
            raise ValueError("Embedding dimension must be aligned to 16 bytes")
        self.model_dim = model_dim

    def __call__(self, final_token_activations: torch.Tensor, all_activations: torch.Tensor,
                 ragged_wrapper) -> torch.Tensor:
        rows = moe_ops.rows_gather(all_activations, ragged_wrapper.meta.last_idx)
        final_token_activations.copy_(rows.view(final_token_activations.shape))
        return final_token_activations


class RaggedTopKGating(DSKernelBase):
    """Softmax router scores, top-k experts per token and each pick's slot inside its expert's group."""
    supported_logit_dtypes = [DtypeEnum.fp16, DtypeEnum.bf16, DtypeEnum.fp32]

    def __init__(self, logit_dtype: DtypeEnum, normalize_scores: bool = False) -> None:
        self.dtype = _check_dtype(logit_dtype, self.supported_logit_dtypes, "logit data type")
        self.normalize = normalize_scores

    def __call__(self, expert_counts: torch.Tensor, scores: torch.Tensor, assignments: torch.Tensor,
                 offsets: torch.Tensor, logits: torch.Tensor, batch=None):
        """logits [T, E] -> scores fp32 [T, k], assignments int32 [T, k], offsets int32 [T, k] (slot inside the
        expert), expert_counts int32 [E]; k is the width of `scores`."""
        k = scores.shape[-1]
        if logits.is_cuda:
            s, a, o, c = moe_ops.topk_gating(logits, k, self.normalize)
        else:
            s, a, _ = moe_ops.topk_gating_reference(logits, k, self.normalize)
            a = a.to(torch.int32)
            E = logits.shape[-1]
            flat = a.reshape(-1).long()
            onehot = torch.nn.functional.one_hot(flat, E)
            o = ((onehot.cumsum(0) - 1) * onehot).sum(-1).view(a.shape).to(torch.int32)
            c = onehot.sum(0).to(torch.int32)
        scores.copy_(s)
        assignments.copy_(a)
        offsets.copy_(o)
        expert_counts.copy_(c)
        return expert_counts, scores, assignments, offsets


class MoEScatter(DSKernelBase):
    """Copy every (token, pick) row to its expert-contiguous position."""
    supported_dtypes = [DtypeEnum.fp16, DtypeEnum.bf16, DtypeEnum.fp32]

    def __init__(self, dtype: DtypeEnum, channels: int) -> None:
        self.dtype = _check_dtype(dtype, self.supported_dtypes)
        if channels % 8 != 0:
            raise ValueError("channels must be divisible by 8")
        self.channels = channels

    def __call__(self, moe_input: torch.Tensor, expert_cumsum: torch.Tensor, mapped_slots: torch.Tensor,
                 activations: torch.Tensor, expert_counts: torch.Tensor, assignments: torch.Tensor,
                 offsets: torch.Tensor):
        """activations [T, H] -> moe_input [T * k, H] grouped by expert, expert_cumsum [E] (inclusive),
        mapped_slots [T, k] (row of each pick in moe_input)."""
        if activations.is_cuda and activations.dtype == torch.bfloat16:
            xs, rows, cum = moe_ops.moe_scatter(activations, assignments, offsets, expert_counts)
        else:
            cum = expert_counts.cumsum(0)
            base = cum - expert_counts
            rows = (base[assignments.long()] + offsets).to(torch.int32)
            xs = torch.empty(rows.numel(), activations.shape[-1], dtype=activations.dtype,
                             device=activations.device)
            k = assignments.shape[-1]
            xs[rows.reshape(-1).long()] = activations.repeat_interleave(k, 0)
        moe_input.copy_(xs.view(moe_input.shape))
        expert_cumsum.copy_(cum.to(expert_cumsum.dtype))
        mapped_slots.copy_(rows.view(mapped_slots.shape))
        return moe_input, expert_cumsum, mapped_slots


class MoEGather(DSKernelBase):
    """layer_output[t] = sum_j scores[t, j] * moe_output[mapped_slots[t, j]]."""
    supported_dtypes = [DtypeEnum.fp16, DtypeEnum.bf16, DtypeEnum.fp32]

    def __init__(self, dtype: DtypeEnum, channels: int, normalize_scores: bool = False) -> None:
        self.dtype = _check_dtype(dtype, self.supported_dtypes)
        if channels % 8 != 0:
            raise ValueError("channels must be divisible by 8")
        self.channels, self.normalize = channels, normalize_scores

    def __call__(self, layer_output: torch.Tensor, moe_output: torch.Tensor, scores: torch.Tensor,
                 mapped_slots: torch.Tensor, expert_counts: torch.Tensor = None) -> torch.Tensor:
        if self.normalize:
            scores = scores / scores.sum(-1, keepdim=True)
        if moe_output.is_cuda and moe_output.dtype == torch.bfloat16:
            out = moe_ops.moe_gather(moe_output, scores.float().contiguous(), mapped_slots)
        else:
            picked = moe_output[mapped_slots.reshape(-1).long()].view(*mapped_slots.shape, -1).float()
            out = (picked * scores.float().unsqueeze(-1)).sum(1).to(moe_output.dtype)
        layer_output.copy_(out.view(layer_output.shape))
        return layer_output
