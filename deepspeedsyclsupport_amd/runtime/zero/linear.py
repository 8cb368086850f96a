"""Memory-efficient linear for ZeRO-3 (reference `runtime/zero/linear.py:43` LinearFunctionForZeroStage3).

torch's `F.linear` saves `weight.t()` — a VIEW of the gathered buffer — for backward, which would keep every
layer's gathered weights alive until backward and defeat partitioning. This autograd function saves the Parameter
itself, so releasing (`p.data = empty`) frees the gathered buffer and the backward pre-hook's re-gather is what the
backward matmuls read.
"""
import types

import torch.nn as nn

from ...ops.linear import LinearFunction

# the training linear of ops/linear.py (saves the Parameter; K-major weight-gradient GEMM for long token dims)
LinearFunctionForZeroStage3 = LinearFunction


def zero3_linear_wrap(input, weight, bias=None):
    return LinearFunctionForZeroStage3.apply(input, weight, bias, getattr(input, "_ds_kmajor", None))


def _zero3_linear_forward(self, x):
    # a producer kernel may have written x's token-contiguous copy for the weight-gradient GEMM (`_ds_kmajor`)
    return LinearFunctionForZeroStage3.apply(x, self.weight, self.bias, getattr(x, "_ds_kmajor", None))


def install_zero3_linear(module: nn.Module):
    """Route every nn.Linear in `module` through LinearFunctionForZeroStage3 (idempotent). Only layers whose forward
    IS `nn.Linear.forward` are patched: a subclass with its own forward (compression layers that apply pruning masks
    or quantisation, tensor-parallel row/column linears that all-reduce or gather) keeps it."""
    n = 0
    for m in module.modules():
        if isinstance(m, nn.Linear) and type(m).forward is nn.Linear.forward and \
                "forward" not in m.__dict__ and not getattr(m, "_ds_zero3_linear", False):
            m.forward = types.MethodType(_zero3_linear_forward, m)
            m._ds_zero3_linear = True
            n += 1
    return n


class LinearModuleForZeroStage3(nn.Linear):
    """nn.Linear whose autograd function saves the Parameter object, not the gathered weight (reference
    `runtime/zero/linear.py:113`): under ZeRO-3 the released weight is not kept alive until backward."""

    def forward(self, input):
        return zero3_linear_wrap(input, self.weight, self.bias)


def print_rank_0(message, debug=False, force=False):
    from ... import comm as dist
    if (debug or force) and (not dist.is_initialized() or dist.get_rank() == 0):
        print(message)

