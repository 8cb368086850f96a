"""Quantizers and the learned top-k mask used by compression training (reference `compression/utils.py`:
TopKBinarizer, SymQuantizer, AsymQuantizer, TernaryQuantizer, BinaryQuantizer — same call signatures
`Q.apply(x, num_bits, min_value=None, max_value=None, num_groups=1)`).

All of them are straight-through estimators: the forward quantises (per group, groups = contiguous slices of the
flattened tensor), the backward passes the gradient through unchanged.
  * symmetric: round(x / s) * s with s = max|x| / (2^(b-1) - 1) per group (or from a static [min, max] range);
  * asymmetric: round((x - lo) / s) * s + lo with s = (hi - lo) / (2^b - 1);
  * ternary (2-bit, "TWN"): {-a, 0, +a}, threshold 0.7 * mean|x|, a = mean |x| over the kept entries;
  * binary (1-bit, "BWN"): sign(x) * mean|x|.
`TopKBinarizer` turns a score tensor into a {0, 1} mask keeping the `threshold` fraction of largest scores; the
gradient reaches the scores unchanged (movement-pruning style), and — with `sigmoid=True` — a learnable threshold
logit receives sum(grad * mask).
"""
import math

import torch


def _groups(x, num_groups):
    n = x.numel()
    g = max(1, min(int(num_groups), n))
    while n % g:
        g -= 1
    return x.reshape(g, n // g)


class TopKBinarizer(torch.autograd.Function):

    @staticmethod
    def forward(ctx, inputs, threshold, sigmoid=False):
        ratio = torch.sigmoid(threshold).item() if sigmoid else float(threshold)
        k = math.ceil(ratio * inputs.numel())
        mask = torch.zeros_like(inputs)
        if k > 0:
            idx = torch.topk(inputs.reshape(-1), k).indices
            mask.view(-1)[idx] = 1.0
        ctx.sigmoid = sigmoid
        ctx.save_for_backward(mask)
        return mask

    @staticmethod
    def backward(ctx, g):
        (mask, ) = ctx.saved_tensors
        gt = (g * mask).sum().view(-1) if ctx.sigmoid else None
        return g, gt, None


class SymQuantizer(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, num_bits, min_value=None, max_value=None, num_groups=1):
        qmax = 2**(num_bits - 1) - 1
        if min_value is not None and max_value is not None:
            s = torch.maximum(min_value.abs(), max_value.abs()).clamp_min(1e-12) / qmax
            return (torch.round(x / s).clamp(-qmax - 1, qmax) * s).to(x.dtype)
        xg = _groups(x.float(), num_groups)
        s = xg.abs().amax(1, keepdim=True).clamp_min(1e-12) / qmax
        return (torch.round(xg / s).clamp(-qmax - 1, qmax) * s).reshape(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None, None


class AsymQuantizer(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, num_bits, min_value=None, max_value=None, num_groups=1):
        levels = 2**num_bits - 1
        if min_value is not None and max_value is not None:
            lo, hi = min_value, max_value
            s = (hi - lo).clamp_min(1e-12) / levels
            return (torch.round((x - lo) / s).clamp(0, levels) * s + lo).to(x.dtype)
        xg = _groups(x.float(), num_groups)
        lo, hi = xg.amin(1, keepdim=True), xg.amax(1, keepdim=True)
        s = (hi - lo).clamp_min(1e-12) / levels
        return (torch.round((xg - lo) / s).clamp(0, levels) * s + lo).reshape(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None, None


class TernaryQuantizer(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, num_bits=2, min_value=None, max_value=None, num_groups=1):
        if min_value is not None or max_value is not None:
            raise ValueError("ternary quantization has no static-range mode")
        xg = _groups(x.float(), num_groups)
        thr = 0.7 * xg.abs().mean(1, keepdim=True)
        keep = (xg.abs() > thr).to(xg.dtype)
        a = (xg.abs() * keep).sum(1, keepdim=True) / keep.sum(1, keepdim=True).clamp_min(1.0)
        return (torch.sign(xg) * keep * a).reshape(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None, None


class BinaryQuantizer(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, num_bits=1, min_value=None, max_value=None, num_groups=1):
        if min_value is not None or max_value is not None:
            raise ValueError("binary quantization has no static-range mode")
        xg = _groups(x.float(), num_groups)
        return (torch.sign(xg) * xg.abs().mean(1, keepdim=True)).reshape(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None, None


def quantizer_for(bits, quantization_type="symmetric"):
    """The straight-through quantizer a weight of `bits` bits uses."""
    if bits == 1:
        return BinaryQuantizer
    if bits == 2:
        return TernaryQuantizer
    return SymQuantizer if quantization_type == "symmetric" else AsymQuantizer
