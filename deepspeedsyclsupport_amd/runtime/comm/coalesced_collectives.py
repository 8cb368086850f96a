"""Batched gradient collectives as free functions (reference `runtime/comm/coalesced_collectives.py:28-145`:
`reduce_scatter_coalesced`, `all_to_all_quant_reduce`). The engine's own gradient path does the same work inside the
flat-group optimizer (`runtime/zero/flat_optimizer.py`, `runtime/zero/zeropp.py`); these entry points serve client
code and tools written against the reference's function names.

`reduce_scatter_coalesced(tensors, group)`: every tensor is cut into `world` chunks of ceil(numel / world) elements;
rank r receives the AVERAGE over the group of chunk r of every tensor. All tensors travel in ONE reduce-scatter: the
send buffer is laid out [world, sum of chunk sizes], filled with one strided copy per tensor (no per-chunk views, no
torch.cat), which is the interleaving that puts the right chunk of every tensor on every rank.
"""
import math
from typing import Dict, List

import torch
from torch import Tensor

from ... import comm as dist
from ...utils.nvtx import instrument_w_nvtx


@instrument_w_nvtx
@torch.no_grad()
def reduce_scatter_coalesced(tensors: List[Tensor], group=None) -> List[Tensor]:
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    sizes = [math.ceil(t.numel() / world) for t in tensors]
    total = sum(sizes)
    ref = tensors[0]
    if len(tensors) == 1 and ref.numel() == world * sizes[0] and ref.is_contiguous():
        send = ref.view(world, sizes[0])  # already in wire layout: reduce in place, no staging buffer
    else:
        send = torch.zeros(world, total, dtype=ref.dtype, device=ref.device)
        off = 0
        for t, n in zip(tensors, sizes):
            flat = t.reshape(-1)
            rows = flat.numel() // n
            if rows:
                send[:rows, off:off + n].copy_(flat[:rows * n].view(rows, n))
            tail = flat.numel() - rows * n
            if tail:
                send[rows, off:off + tail].copy_(flat[rows * n:])
            off += n
    send.div_(world)  # pre-divide: the sum of the scaled chunks is the group average
    out = torch.empty(total, dtype=ref.dtype, device=ref.device)
    dist.reduce_scatter_tensor(out, send.reshape(-1), group=group)
    res, off = [], 0
    for t, n in zip(tensors, sizes):
        valid = max(0, min(n, t.numel() - rank * n))  # the last ranks' chunks may be partly (or wholly) padding
        res.append(out.narrow(0, off, valid))
        off += n
    return res


@instrument_w_nvtx
@torch.no_grad()
def all_to_all_quant_reduce(tensors: List[Tensor], groups: Dict = None) -> List[Tensor]:
    """qgZ gradient reduction (reference `coalesced_collectives.py:30-70`): 1-D tensors take the plain batched
    reduce-scatter; matrices are exchanged as int8 blocks through one all-to-all and summed by the fused
    dequantise-reduce kernel (`runtime/zero/zeropp.py`). One xGMI node is a single level: `groups` may carry the
    group to use under the key "world" (default: all ranks); the reference's two-level intra / inter-node split is
    not needed on a fully connected node; when `groups` is the reference's table (`local_<node>`, `global_<local
    index>`, as `parallel.groups._get_local_all_to_all_group()` builds it) and it spans several nodes, the exchange runs
    in two levels (`zeropp.quantized_reduce_scatter_2level`)."""
    from ..zero.zeropp import quantized_reduce_scatter, quantized_reduce_scatter_2level
    groups = groups or {}
    group = groups.get("world")
    world = dist.get_world_size(group)
    # the reference's group table (`local_<node>` / `global_<local index>`): two levels when it spans several nodes
    from ..zero.zeropp import levels_from_table
    levels = levels_from_table(groups)
    out: List[Tensor] = [None] * len(tensors)
    for i, t in enumerate(tensors):
        if t.dim() == 1 or t.numel() % (world * 64):
            out[i] = reduce_scatter_coalesced([t], group)[0]
            continue
        seg = t.numel() // world
        buf = torch.empty(seg, dtype=torch.float32, device=t.device)
        if levels is not None:
            quantized_reduce_scatter_2level(buf, t.reshape(-1), *levels)
        else:
            quantized_reduce_scatter(buf, t.reshape(-1), group)
        out[i] = buf.div_(world).to(t.dtype)
    return out
