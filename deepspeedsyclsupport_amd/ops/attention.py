"""Attention dispatch for training and prefill.

On MI355X (bf16, head dim 128, no explicit mask / dropout) the forward runs the in-tree CDNA4 flash-attention kernel
(`csrc/attn/flash_fwd.hip`: MFMA 32x32x16, swapped QK^T with in-register online softmax, transposed-LDS V reads).
Its output memory is laid out [B, S, H, D], so the caller's `o.transpose(1, 2).reshape(B, S, H*D)` is free. The
backward reuses the memory-efficient SDPA backward kernel, fed with our (O, LSE) pair — the kernel's contract is
exactly (q, k, v, o, natural-log LSE [B,H,S]) (`tools/probe_attn_bwd.py` checks the interchange on the GPU).

Everything else (other head dims, masks, dropout, fp16/fp32, host tensors) goes through torch SDPA with the
memory-efficient backend preferred (measured on MI355X: 451 TF fwd+bwd causal at B4·H32·S4096·D128 vs 243 TF for
SDPA-flash; `profiles/probe_gpu_r1.log`).
"""
import os

import torch
import torch.nn.functional as F

try:
    from torch.nn.attention import SDPBackend, sdpa_kernel
    _PREF = [SDPBackend.EFFICIENT_ATTENTION, SDPBackend.FLASH_ATTENTION, SDPBackend.MATH]
except Exception:  # pragma: no cover
    sdpa_kernel = None

_USE_FLASH = os.environ.get("DS_FLASH_ATTN", "1") != "0"


def _sdpa(q, k, v, causal, scale, attn_mask=None, dropout_p=0.0):
    gqa = q.shape[1] != k.shape[1]
    kw = dict(is_causal=causal and attn_mask is None, scale=scale, attn_mask=attn_mask, dropout_p=dropout_p)
    if gqa:
        kw["enable_gqa"] = True
    if q.is_cuda and sdpa_kernel is not None:
        with sdpa_kernel(_PREF, set_priority=True):
            return F.scaled_dot_product_attention(q, k, v, **kw)
    if gqa:
        rep = q.shape[1] // k.shape[1]
        k = k.repeat_interleave(rep, dim=1)
        v = v.repeat_interleave(rep, dim=1)
        kw.pop("enable_gqa")
    return F.scaled_dot_product_attention(q, k, v, **kw)


_ZEROS = {}


def _zero_seed(device):
    z = _ZEROS.get(device)
    if z is None:
        z = _ZEROS[device] = torch.zeros((), dtype=torch.int64, device=device)
    return z


class FlashAttnFunc(torch.autograd.Function):
    """Forward: gfx950 flash kernel (O, LSE). Backward: efficient-attention backward on that (O, LSE)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        from .native import hip_ops
        need_grad = any(t.requires_grad for t in (q, k, v))
        o, lse = hip_ops().flash_fwd(q, k, v, bool(causal), float(scale), need_grad)
        if need_grad:
            ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = bool(causal), float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        hq, hk = q.shape[1], k.shape[1]
        rep = hq // hk
        ke = k.repeat_interleave(rep, dim=1) if rep > 1 else k
        ve = v.repeat_interleave(rep, dim=1) if rep > 1 else v
        z = _zero_seed(q.device)  # no dropout: philox seed/offset unused
        do = do if do.stride(-1) == 1 else do.contiguous()
        dq, dk, dv, _ = torch.ops.aten._scaled_dot_product_efficient_attention_backward(
            do, q, ke, ve, None, o, lse, z, z, 0.0, [True, True, True, False], ctx.causal, scale=ctx.scale)
        if rep > 1:
            B, _, S, D = dk.shape
            dk = dk.view(B, hk, rep, S, D).sum(2)
            dv = dv.view(B, hk, rep, S, D).sum(2)
        return dq, dk, dv, None, None


def flash_supported(q, k, v, attn_mask=None, dropout_p=0.0):
    return (_USE_FLASH and q.is_cuda and attn_mask is None and dropout_p == 0.0 and q.dtype == torch.bfloat16
            and k.dtype == torch.bfloat16 and v.dtype == torch.bfloat16 and q.shape[-1] == 128
            and k.shape[-1] == 128 and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1
            and q.shape[1] % k.shape[1] == 0 and all(s % 8 == 0 for t in (q, k, v) for s in t.stride()[:3]))


def attention(q, k, v, causal=True, softmax_scale=None, attn_mask=None, dropout_p=0.0):
    """q [B, Hq, S, D], k/v [B, Hk, S, D] -> o [B, Hq, S, D]."""
    if flash_supported(q, k, v, attn_mask, dropout_p):
        scale = softmax_scale if softmax_scale is not None else q.shape[-1]**-0.5
        return FlashAttnFunc.apply(q, k, v, causal, scale)
    return _sdpa(q, k, v, causal, softmax_scale, attn_mask, dropout_p)
