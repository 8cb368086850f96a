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


def kmajor_wanted(rows, dtype):
    """Should a producer of a [rows, n] linear operand also write its token-contiguous copy? (same test as the
    weight-gradient GEMM's, so a copy is only made where it will be used)"""
    return _ENABLED and rows >= KMAJOR_MIN_ROWS and rows % 8 == 0 and dtype in (torch.bfloat16, torch.float16)


STATS = {"kmajor_from_producer": 0, "kmajor_transposed": 0}  # how the weight-gradient operands were obtained


def _kmajor_of(t2d, given, Tp):
    """The [n, Tp] token-contiguous copy of t2d [T, n]: the one its producer wrote (`given`) or a transpose pass."""
    if given is not None and given.shape == (t2d.shape[1], Tp) and given.dtype == t2d.dtype:
        STATS["kmajor_from_producer"] += 1
        return given
    from .native import hip_ops
    STATS["kmajor_transposed"] += 1
    return hip_ops().transpose16(_rows16(t2d), Tp)


def weight_grad(go2d, x2d, go_kmajor=None, x_kmajor=None):
    """[T, out], [T, in] -> dW [out, in]. The K-major copies are zero-padded to a multiple of 256 tokens (e.g. the
    LM head's 32760 shifted tokens -> 32768: measured 7.6 ms -> 5.0 ms for that GEMM). `x2d` may be None when the
    forward kept only `x_kmajor`."""
    T = go2d.shape[0]
    if x_kmajor is not None or _kmajor_ok(go2d, x2d):
        Tp = -(-T // 256) * 256
        got = _kmajor_of(go2d, go_kmajor, Tp)                                    # [out, Tp]
        if x2d is None:
            STATS["kmajor_from_producer"] += 1
        xt = x_kmajor if x2d is None else _kmajor_of(x2d, x_kmajor, Tp)          # [in, Tp]
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
    """y = x W^T + b. `x_kmajor` ([in, Tp], written by x's producer) replaces x in what is kept for backward: the
    weight gradient is its only use, so the row-major activation is not kept alive at all."""

    @staticmethod
    def forward(ctx, x, weight, bias=None, x_kmajor=None):
        if x_kmajor is not None:
            ctx.save_for_backward(x_kmajor, weight, bias)
            ctx.kmajor_saved = True
        else:
            ctx.save_for_backward(x, weight, bias)
            ctx.kmajor_saved = False
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
            go_t = getattr(go, "_ds_kmajor", None)  # written by the gradient's producer kernel, if it makes one
            if ctx.kmajor_saved:
                gw = weight_grad(go2, None, go_t, x.to(go.dtype))
            else:
                gw = weight_grad(go2, x.reshape(-1, x.shape[-1]).to(go.dtype), go_t)
        if bias is not None and ctx.needs_input_grad[2]:
            gb = go2.sum(0)
        return gx, gw, gb, None


def linear(x, weight, bias=None):
    return LinearFunction.apply(x, weight, bias, getattr(x, "_ds_kmajor", None))
