"""Attention dispatch for training and prefill.

Order of preference on MI355X: the in-tree CDNA4 flash-attention kernel (`ds_hip_ops.flash_attn_*`, once built),
else torch SDPA with the memory-efficient backend preferred (measured on MI355X: 451 TF fwd+bwd causal at
B4·H32·S4096·D128 vs 243 TF for SDPA-flash; `profiles/probe_gpu.log`). Host tensors use the math backend.
"""
import torch
import torch.nn.functional as F

try:
    from torch.nn.attention import SDPBackend, sdpa_kernel
    _PREF = [SDPBackend.EFFICIENT_ATTENTION, SDPBackend.FLASH_ATTENTION, SDPBackend.MATH]
except Exception:  # pragma: no cover
    sdpa_kernel = None


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


def attention(q, k, v, causal=True, softmax_scale=None, attn_mask=None, dropout_p=0.0):
    """q [B, Hq, S, D], k/v [B, Hk, S, D] -> o [B, Hq, S, D]."""
    return _sdpa(q, k, v, causal, softmax_scale, attn_mask, dropout_p)
