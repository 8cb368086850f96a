"""Channels-last (NHWC) bias-add fusions for diffusion UNet / VAE inference (reference `op_builder/spatial_inference.py`,
`csrc/spatial/csrc/opt_bias_add.cu` + `pt_binding.cpp:109-111`: `nhwc_bias_add`, `nhwc_bias_add_add`,
`nhwc_bias_add_bias_add`).

The activation is [N, H, W, C] with C innermost (a channels-last conv output, `memory_format=torch.channels_last`
viewed as NHWC, or an [N, HW, C] token tensor); the biases are per channel. Device tensors use ONE gfx950 kernel
(16-B vectors over channels, fp32 math); host tensors use the same formula in PyTorch.
"""
import torch

from ..native import hip_ops


def _nhwc(t):
    """[N, C, H, W] channels_last tensors are viewed as contiguous [N, H, W, C]."""
    if t.dim() == 4 and not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1), True
    return t, False


def _run(activation, bias, other=None, other_bias=None):
    x, was_cl = _nhwc(activation)
    o = _nhwc(other)[0] if other is not None else None
    if x.is_cuda and x.is_contiguous() and x.shape[-1] % 8 == 0 and (o is None or o.is_contiguous()):
        y = hip_ops().bias_add2(x, bias.contiguous(), o, None if other_bias is None else other_bias.contiguous())
    else:
        y = x + bias
        if o is not None:
            y = y + o
        if other_bias is not None:
            y = y + other_bias
    return y.permute(0, 3, 1, 2) if was_cl else y


def nhwc_bias_add(activation, bias):
    return _run(activation, bias)


def nhwc_bias_add_add(activation, bias, other):
    return _run(activation, bias, other)


def nhwc_bias_add_bias_add(activation, bias, other, other_bias):
    return _run(activation, bias, other, other_bias)


__all__ = ["nhwc_bias_add", "nhwc_bias_add_add", "nhwc_bias_add_bias_add"]
