"""Attention dispatch for training and prefill.

On MI355X (bf16, head dim 128, no explicit mask / dropout) both passes run in-tree CDNA4 kernels:
 * forward `csrc/attn/flash_fwd.hip` (MFMA 32x32x16, swapped QK^T with in-register online softmax, transposed-LDS V
   reads). Its output memory is laid out [B, S, H, D], so the caller's `o.transpose(1, 2).reshape(B, S, H*D)` is free;
 * backward `csrc/attn/flash_bwd.hip`: one workgroup per 256 keys of one (batch, kv head) sweeping every query head
   of the GQA group (no repeat_interleave of K/V, no dK/dV reduction), P recomputed from the forward's LSE, dQ by
   f32 atomics. dq/dk/dv come back in the same [B, S, H, D] memory layout.

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


class FlashAttnFunc(torch.autograd.Function):
    """Forward and backward on the gfx950 flash kernels (csrc/attn/flash_{fwd,bwd}.hip)."""

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
        from .native import hip_ops
        q, k, v, o, lse = ctx.saved_tensors
        if do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]) or do.data_ptr() % 16:
            do = do.contiguous()
        dq, dk, dv = hip_ops().flash_bwd(q, k, v, o, lse, do, ctx.scale, 1 if ctx.causal else 0)
        return dq, dk, dv, None, None


def flash_supported(q, k, v, attn_mask=None, dropout_p=0.0):
    return (_USE_FLASH and q.is_cuda and attn_mask is None and dropout_p == 0.0 and q.dtype == torch.bfloat16
            and k.dtype == torch.bfloat16 and v.dtype == torch.bfloat16 and q.shape[-1] == 128
            and k.shape[-1] == 128 and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1
            and q.shape[1] % k.shape[1] == 0 and all(s % 8 == 0 for t in (q, k, v) for s in t.stride()[:3])
            and (not any(t.requires_grad for t in (q, k, v)) or q.shape[2] == k.shape[2]))


def attention(q, k, v, causal=True, softmax_scale=None, attn_mask=None, dropout_p=0.0):
    """q [B, Hq, S, D], k/v [B, Hk, S, D] -> o [B, Hq, S, D]."""
    if flash_supported(q, k, v, attn_mask, dropout_p):
        scale = softmax_scale if softmax_scale is not None else q.shape[-1]**-0.5
        return FlashAttnFunc.apply(q, k, v, causal, scale)
    return _sdpa(q, k, v, causal, softmax_scale, attn_mask, dropout_p)
