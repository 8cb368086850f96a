"""Tensor-parallel building blocks used by AutoTP and kernel injection (reference `module_inject/layers.py:16-160`).

Column-parallel layers (`LinearLayer`) hold a row slice of W and need no communication; row-parallel layers
(`LinearAllreduce`) hold a column slice and sum partial outputs with one RCCL all-reduce (bias added once, after it).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist


class LinearAllreduce(nn.Module):

    def __init__(self, weight, bias=None, mp_group=None):
        super().__init__()
        self.weight = weight if isinstance(weight, nn.Parameter) else nn.Parameter(weight, requires_grad=False)
        self.bias = bias if (bias is None or isinstance(bias, nn.Parameter)) else nn.Parameter(bias,
                                                                                             requires_grad=False)
        self.mp_group = mp_group

    # local shapes, as the nn.Linear this stands in for would report them
    in_features = property(lambda self: self.weight.shape[1])
    out_features = property(lambda self: self.weight.shape[0])

    def forward(self, input):
        out = F.linear(input, self.weight)
        if self.mp_group is not None and dist.get_world_size(self.mp_group) > 1:
            dist.inference_all_reduce(out, group=self.mp_group)
        if self.bias is not None:
            out = out + self.bias
        return out


class LmHeadLinearAllreduce(nn.Module):
    """Row-parallel LM head: each rank holds a hidden-dim slice; input is sliced to match, logits all-reduced."""

    def __init__(self, weight, rank, world_size, bias=None, mp_group=None):
        super().__init__()
        self.weight = nn.Parameter(weight, requires_grad=False)
        self.bias = None if bias is None else nn.Parameter(bias, requires_grad=False)
        self.rank, self.world_size, self.mp_group = rank, world_size, mp_group

    def forward(self, input):
        n = input.shape[-1] // self.world_size
        out = F.linear(input[..., self.rank * n:(self.rank + 1) * n], self.weight)
        if self.mp_group is not None and self.world_size > 1:
            dist.inference_all_reduce(out, group=self.mp_group)
        if self.bias is not None:
            out = out + self.bias
        return out


class LinearLayer(nn.Module):

    def __init__(self, weight_shape=None, dtype=torch.bfloat16, weight=None, bias=None):
        super().__init__()
        if weight is None:
            weight = torch.empty(weight_shape, dtype=dtype)
        self.weight = weight if isinstance(weight, nn.Parameter) else nn.Parameter(weight, requires_grad=False)
        self.bias = bias if (bias is None or isinstance(bias, nn.Parameter)) else nn.Parameter(bias,
                                                                                             requires_grad=False)

    in_features = property(lambda self: self.weight.shape[1])
    out_features = property(lambda self: self.weight.shape[0])

    def forward(self, input):
        return F.linear(input, self.weight, self.bias)


class Normalize(nn.Module):

    def __init__(self, dim=None, dtype=torch.float, eps=1e-5, weight=None, bias=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(weight if weight is not None else torch.ones(dim, dtype=dtype))
        self.bias = nn.Parameter(bias if bias is not None else torch.zeros(dim, dtype=dtype))

    def forward(self, input):
        from ..ops.transformer.functional import layer_norm
        return layer_norm(input, self.weight, self.bias, self.eps)


class RMSNormalize(nn.Module):

    def __init__(self, dim=None, dtype=torch.float, eps=1e-5, weight=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(weight if weight is not None else torch.ones(dim, dtype=dtype))

    def forward(self, hidden_states):
        from ..ops.transformer.functional import rms_norm
        return rms_norm(hidden_states, self.weight, self.eps)


class EmbeddingLayer(nn.Module):

    def __init__(self, weight_shape=None, dtype=torch.bfloat16, weight=None, bias=None):
        super().__init__()
        self.weight = nn.Parameter(weight if weight is not None else torch.empty(weight_shape, dtype=dtype))

    def forward(self, input):
        return F.embedding(input, self.weight)


class OPTEmbedding(EmbeddingLayer):
    """Learned positions with OPT's offset of 2, computed from the attention mask."""

    def __init__(self, weight_shape=None, weight=None, bias=None):
        super().__init__(weight_shape, weight=weight)
        self.offset = 2

    def forward(self, attention_mask, past_key_values_length: int = 0):
        attention_mask = attention_mask.long()
        positions = (torch.cumsum(attention_mask, dim=1).type_as(attention_mask) * attention_mask).long() - 1
        positions = positions[:, past_key_values_length:]
        return super().forward(positions + self.offset)
