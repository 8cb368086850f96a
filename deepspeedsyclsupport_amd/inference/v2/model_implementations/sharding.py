"""Tensor-parallel slicing rules of the inference v2 models (reference
`inference/v2/model_implementations/sharding/{types,utils,qkv,attn_out,mlp,embedding,unembed,attn}.py`).

The rules, for `num_shards` ranks:
  * attention: query heads are dealt out in contiguous runs; key / value heads likewise when there are at least as
    many as ranks, otherwise a rank holds the one kv head its query heads attend with (replicated across the ranks
    of a group);
  * QKV weight rows follow the heads; the attention output projection splits its input columns the same way;
  * MLP: first projection by rows of the intermediate dim (gate and up halves each), second by columns;
  * embedding: by columns of the hidden dim; un-embedding (LM head): by vocabulary rows.
Dimensions that do not divide are split at multiples of `granularity`, earlier ranks taking the larger share.
"""
from enum import Enum
from typing import Optional, Tuple

import torch

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`

DEFAULT_SHARD_GRANULARITY = 32


class ShardingType(Enum):
    OUTER_DIMENSION = 0   # rows of a [out, in] weight (and the only dim of its bias)
    INNER_DIMENSION = 1   # columns of a [out, in] weight (its bias stays whole)


def get_shard_endpoints(dim_size: int, shard_rank: int, num_shards: int,
                        granularity: int = DEFAULT_SHARD_GRANULARITY) -> Tuple[int, int]:
    if dim_size % granularity:
        raise ValueError(f"dimension {dim_size} is not a multiple of the shard granularity {granularity}")
    units = dim_size // granularity
    base, extra = divmod(units, num_shards)
    lo = shard_rank * base + min(shard_rank, extra)
    hi = lo + base + (1 if shard_rank < extra else 0)
    return lo * granularity, hi * granularity


def shard_param(param: Optional[torch.Tensor], shard_mode: ShardingType, shard_rank: int, num_shards: int,
                num_concatenated_matrices: int = 1, granularity: int = DEFAULT_SHARD_GRANULARITY,
                bias_dims: int = 1) -> Optional[torch.Tensor]:
    """Slice a weight ([.., out, in]) or bias ([.., out], `bias_dims` trailing dims or fewer) for one rank. A tensor
    made of `num_concatenated_matrices` matrices stacked along `out` (gate | up) is sliced per matrix."""
    if param is None or num_shards == 1:
        return param
    is_bias = param.dim() <= bias_dims
    if shard_mode == ShardingType.INNER_DIMENSION:
        if is_bias:
            return param
        lo, hi = get_shard_endpoints(param.shape[-1], shard_rank, num_shards, granularity)
        return param[..., lo:hi]
    dim = param.dim() - 1 if is_bias else param.dim() - 2
    per = param.shape[dim] // num_concatenated_matrices
    lo, hi = get_shard_endpoints(per, shard_rank, num_shards, granularity)
    pieces = [param.narrow(dim, m * per + lo, hi - lo) for m in range(num_concatenated_matrices)]
    return pieces[0] if len(pieces) == 1 else torch.cat(pieces, dim=dim)


def get_local_heads(shard_rank: int, num_shards: int, n_heads_q: int, n_heads_kv: Optional[int] = None):
    """(query heads, kv heads) held by a rank."""
    n_heads_kv = n_heads_kv or n_heads_q
    if n_heads_q % num_shards:
        raise ValueError(f"{n_heads_q} query heads do not divide over {num_shards} ranks")
    if n_heads_kv >= num_shards:
        if n_heads_kv % num_shards:
            raise ValueError(f"{n_heads_kv} kv heads do not divide over {num_shards} ranks")
        return n_heads_q // num_shards, n_heads_kv // num_shards
    return n_heads_q // num_shards, 1


def _kv_range(shard_rank, num_shards, n_heads_q, n_heads_kv):
    if n_heads_kv >= num_shards:
        per = n_heads_kv // num_shards
        return shard_rank * per, (shard_rank + 1) * per
    group = n_heads_q // n_heads_kv
    kv = (shard_rank * (n_heads_q // num_shards)) // group
    return kv, kv + 1


def shard_qkv_param(param: Optional[torch.Tensor], shard_rank: int, num_shards: int, head_size: int,
                    n_heads_q: Optional[int] = None, n_heads_kv: Optional[int] = None) -> Optional[torch.Tensor]:
    """Fused [q | k | v] weight ([(Hq + 2 Hkv) * D, in]) or bias -> this rank's [q | k | v]."""
    if param is None or num_shards == 1:
        return param
    if n_heads_q is None:
        n_heads_q = param.shape[0] // (3 * head_size)
    n_heads_kv = n_heads_kv or n_heads_q
    get_local_heads(shard_rank, num_shards, n_heads_q, n_heads_kv)
    q, k, v = param.split([n_heads_q * head_size, n_heads_kv * head_size, n_heads_kv * head_size], dim=0)
    per = n_heads_q // num_shards
    klo, khi = _kv_range(shard_rank, num_shards, n_heads_q, n_heads_kv)
    return torch.cat([q[shard_rank * per * head_size:(shard_rank + 1) * per * head_size],
                      k[klo * head_size:khi * head_size], v[klo * head_size:khi * head_size]], dim=0)


def qkv_out_features(in_features: int, shard_rank: int, num_shards: int, head_size: int,
                     n_heads_q: Optional[int] = None, n_heads_kv: Optional[int] = None) -> int:
    n_heads_q = n_heads_q or in_features // head_size
    hq, hk = get_local_heads(shard_rank, num_shards, n_heads_q, n_heads_kv)
    return (hq + 2 * hk) * head_size


def shard_attn_out_param(param: Optional[torch.Tensor], shard_rank: int, num_shards: int, head_size: int,
                         n_heads_q: Optional[int] = None, n_heads_kv: Optional[int] = None):
    """Output projection [out, Hq * D]: columns of this rank's query heads; the bias goes to rank 0 only (the
    all-reduce then adds it once)."""
    if param is None or num_shards == 1:
        return param
    if param.dim() == 1:
        return param if shard_rank == 0 else None
    n_heads_q = n_heads_q or param.shape[1] // head_size
    per = n_heads_q // num_shards
    return param[:, shard_rank * per * head_size:(shard_rank + 1) * per * head_size]


def attn_out_in_features(out_features: int, shard_rank: int, num_shards: int, head_size: int,
                         n_heads_q: Optional[int] = None, n_heads_kv: Optional[int] = None) -> int:
    n_heads_q = n_heads_q or out_features // head_size
    return get_local_heads(shard_rank, num_shards, n_heads_q, n_heads_kv)[0] * head_size


def shard_mlp_1_param(param: Optional[torch.Tensor], shard_rank: int, num_shards: int, gated: bool = False,
                      is_moe: bool = False) -> Optional[torch.Tensor]:
    return shard_param(param, ShardingType.OUTER_DIMENSION, shard_rank, num_shards,
                       num_concatenated_matrices=2 if gated else 1, bias_dims=2 if is_moe else 1)


def shard_mlp_2_param(param: Optional[torch.Tensor], shard_rank: int, num_shards: int,
                      is_moe: bool = False) -> Optional[torch.Tensor]:
    bias_dims = 2 if is_moe else 1
    if param is not None and param.dim() <= bias_dims:
        return param if shard_rank == 0 else None
    return shard_param(param, ShardingType.INNER_DIMENSION, shard_rank, num_shards, bias_dims=bias_dims)


def sharded_intermediate_dim(intermediate_size: int, num_shards: int, shard_rank: int) -> int:
    lo, hi = get_shard_endpoints(intermediate_size, shard_rank, num_shards)
    return hi - lo


def shard_embedding_param(param: torch.Tensor, shard_rank: int, num_shards: int) -> torch.Tensor:
    return shard_param(param, ShardingType.INNER_DIMENSION, shard_rank, num_shards)


def sharded_embedding_dim(embedding_size: int, shard_rank: int, num_shards: int) -> int:
    lo, hi = get_shard_endpoints(embedding_size, shard_rank, num_shards)
    return hi - lo


def shard_unembed_param(param: torch.Tensor, shard_rank: int, num_shards: int) -> torch.Tensor:
    return shard_param(param, ShardingType.OUTER_DIMENSION, shard_rank, num_shards, granularity=1)


def sharded_unembed_dim(vocab_size: int, shard_rank: int, num_shards: int) -> int:
    lo, hi = get_shard_endpoints(vocab_size, shard_rank, num_shards, granularity=1)
    return hi - lo
