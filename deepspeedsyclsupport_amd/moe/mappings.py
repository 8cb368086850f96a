"""Token mappings between a tensor-parallel non-expert part and experts that are not tensor parallel (reference
`moe/mappings.py:27-106`).

With Megatron-style tensor parallelism every TP rank of a replica holds the same tokens. Experts that are not
themselves tensor parallel would process each token TP times, so before the expert all-to-all every TP rank keeps
only its 1/TP share of the capacity slots (`drop_tokens`, a view: no traffic), and after the return all-to-all the
shares are all-gathered back (`gather_tokens`) for the tensor-parallel layers that follow. Each is the other's
backward. On an xGMI node this also divides the all-to-all volume by TP.
"""
import torch

from .. import comm as dist
from ..parallel import groups


def _tp():
    """(world size, rank, group) of the tensor-parallel group of the installed mpu; (1, 0, None) without one."""
    mpu = groups.mpu
    if mpu is None:
        return 1, 0, None
    for pre in ("get_tensor_model_parallel", "get_slice_parallel", "get_model_parallel"):
        if hasattr(mpu, pre + "_world_size"):
            return (getattr(mpu, pre + "_world_size")(), getattr(mpu, pre + "_rank")(), getattr(mpu, pre + "_group")())
    return 1, 0, None


def tensor_parallel_world_size():
    return _tp()[0]


def _gather(x, dim):
    world, rank, group = _tp()
    x = x.contiguous()
    if dim == 0:
        out = torch.empty((world * x.shape[0], ) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x, group=group)
    return torch.cat(parts, dim=dim)


def _drop(x, dim):
    world, rank, _ = _tp()
    assert x.shape[dim] % world == 0, \
        f"input dimension {dim} ({x.shape[dim]}) is not divisible by tensor parallel world size ({world})"
    n = x.shape[dim] // world
    return x.narrow(dim, rank * n, n)


class _GatherTokens(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, dim):
        ctx.dim = dim
        return _gather(x, dim)

    @staticmethod
    def backward(ctx, g):
        return _drop(g, ctx.dim), None


class _DropTokens(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, dim):
        ctx.dim = dim
        return _drop(x, dim)

    @staticmethod
    def backward(ctx, g):
        return _gather(g, ctx.dim), None


def gather_tokens(input_, dim=0):
    if tensor_parallel_world_size() == 1:
        return input_
    return _GatherTokens.apply(input_, dim)


def drop_tokens(input_, dim=0):
    if tensor_parallel_world_size() == 1:
        return input_
    return _DropTokens.apply(input_, dim)
