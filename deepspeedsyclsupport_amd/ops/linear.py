"""Training linear layer with a K-major weight-gradient GEMM.

`dW = dY^T X` contracts over the token dimension. Read straight from the [T, out] / [T, in] activations both GEMM
operands are MN-major, a layout the library GEMMs run at ~1.0-1.1 PF/s on MI355X for the Llama-7B shapes
(T = 32768); with K-major operands the same GEMM runs at ~1.4-1.5 PF/s (`profiles/wgrad_gemm_layouts_r2.jsonl`).
So for long token dimensions the backward first streams dY and X through the HBM-speed transpose kernel
(`csrc/act/transpose.hip`) and then issues the K-major GEMM. The function also saves the Parameter (not a view of
it), so under ZeRO-3 a released gathered weight is not kept alive by autograd (reference
`runtime/zero/linear.py:43` LinearFunctionForZeroStage3).
"""
import os

import torch
import torch.nn.functional as F

KMAJOR_MIN_ROWS = int(os.environ.get("DS_WGRAD_KMAJOR_MIN_ROWS", "8192"))
_ENABLED = os.environ.get("DS_WGRAD_KMAJOR", "1") != "0"
_DGRAD_ENABLED = os.environ.get("DS_DGRAD_KMAJOR", "1") != "0"


def _kmajor_ok(go, x):
    T = go.shape[0]
    return (_ENABLED and go.is_cuda and T >= KMAJOR_MIN_ROWS and go.dtype in (torch.bfloat16, torch.float16)
            and x.dtype == go.dtype and T % 8 == 0 and go.shape[1] % 8 == 0 and x.shape[1] % 8 == 0)


def _rows16(t):
    if t.stride(1) != 1 or t.stride(0) % 8 or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def weight_grad(go2d, x2d):
    """[T, out], [T, in] -> dW [out, in]. The K-major copies are zero-padded to a multiple of 256 tokens (e.g. the
    LM head's 32760 shifted tokens -> 32768: measured 7.6 ms -> 5.0 ms for that GEMM)."""
    if _kmajor_ok(go2d, x2d):
        from .native import hip_ops
        h = hip_ops()
        Tp = -(-go2d.shape[0] // 256) * 256
        got = h.transpose16(_rows16(go2d), Tp)   # [out, Tp]
        xt = h.transpose16(_rows16(x2d), Tp)     # [in, Tp]
        return torch.mm(got, xt.t())
    return go2d.t().mm(x2d)


def input_grad(go2d, weight):
    """[T, out] . W [out, in] -> dX [T, in]. Read row-major, W is an MN-major B operand; for long token dimensions
    a K-major copy W^T [in, out] (one HBM-speed transpose of the weight, ~0.04 ms for a 7B layer's QKV) turns the
    product into the TN layout of the forward GEMMs."""
    if _DGRAD_ENABLED and _kmajor_ok(go2d, weight) and weight.dim() == 2 and weight.stride(1) == 1:
        from .native import hip_ops
        wt = hip_ops().transpose16(_rows16(weight))   # [in, out]
        return torch.mm(go2d, wt.t())
    return go2d.mm(weight)


class LinearFunction(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, weight, bias=None):
        ctx.save_for_backward(x, weight, bias)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, go):
        # under autocast the forward GEMM ran in the autocast dtype while x / weight were saved as given: the
        # backward products run in the gradient's dtype
        x, weight, bias = ctx.saved_tensors
        gx = gw = gb = None
        go2 = go.reshape(-1, go.shape[-1])
        if ctx.needs_input_grad[0]:
            gx = input_grad(go2, weight.to(go.dtype)).view(*go.shape[:-1], weight.shape[1])
        if ctx.needs_input_grad[1]:
            gw = weight_grad(go2, x.reshape(-1, x.shape[-1]).to(go.dtype))
        if bias is not None and ctx.needs_input_grad[2]:
            gb = go2.sum(0)
        return gx, gw, gb


def linear(x, weight, bias=None):
    return LinearFunction.apply(x, weight, bias)
