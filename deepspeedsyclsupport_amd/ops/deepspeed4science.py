"""DS4Science Evoformer attention (reference `ops/deepspeed4science/evoformer_attn.py:14-106`):
out = softmax(Q K^T / sqrt(D) + bias1 + bias2) V over [B, N, S, H, D] tensors (MSA row/column attention in
AlphaFold-style models), bias1 = per-key mask bias [B, N, 1, 1, S], bias2 = pair bias [B, 1, H, S, S]; gradients
flow to Q, K, V and both biases.

On MI355X (bf16/fp16, head dim 32 or 64) both passes run the fused kernel `csrc/attn/flash_small.hip`
(`ops/flash_small.py`): B*N folds into one z axis, bias1 is read per key, bias2 is shared by the N rows of a batch
(b2_div = N) and its gradient is summed over them in-kernel — no [B, N, H, S, S] tensor is materialised in either
pass (the reference's CUTLASS kernels, `csrc/deepspeed4science/evoformer_attn/attention_*.cu`, have the same
contract). Host tensors, fp32 and other head dims use torch SDPA with the summed bias.
"""
import math

import torch
import torch.nn.functional as F

from . import flash_small as FS

__path__ = []  # lets the reference's per-class sub-paths resolve through `_import_paths`


def _check_shapes(Q, biases):
    B, N, S, H, D = Q.shape
    if biases[0] is not None:
        assert tuple(biases[0].shape) == (B, N, 1, 1, S), "bias1 shape is incorrect"
    if biases[1] is not None:
        assert tuple(biases[1].shape) == (B, 1, H, S, S), "bias2 shape is incorrect"


def _sdpa_path(Q, K, V, biases):
    B, N, S, H, D = Q.shape
    q = Q.permute(0, 1, 3, 2, 4).reshape(B * N, H, S, D)
    k = K.permute(0, 1, 3, 2, 4).reshape(B * N, H, S, D)
    v = V.permute(0, 1, 3, 2, 4).reshape(B * N, H, S, D)
    bias = None
    if biases[0] is not None:
        bias = biases[0].expand(B, N, H, S, S)
    if biases[1] is not None:
        b2 = biases[1].expand(B, N, H, S, S)
        bias = b2 if bias is None else bias + b2
    if bias is not None:
        bias = bias.reshape(B * N, H, S, S).to(q.dtype)
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale=1.0 / math.sqrt(D))
    return o.view(B, N, H, S, D).permute(0, 1, 3, 2, 4)


def _kernel_path(Q, K, V, biases):
    B, N, S, H, D = Q.shape
    q, k, v = (t.reshape(B * N, S, H, D) for t in (Q, K, V))
    b1 = biases[0].reshape(B * N, S).to(Q.dtype) if biases[0] is not None else None
    b2 = biases[1].reshape(B, H, S, S).to(Q.dtype) if biases[1] is not None else None
    o = FS.flash_small(q, k, v, b1, b2, b2_div=N, scale=1.0 / math.sqrt(D))
    return o.view(B, N, S, H, D)


def DS4Sci_EvoformerAttention(Q, K, V, biases):
    assert Q.dim() == 5, "expected [B, N, S, H, D]"
    biases = list(biases) + [None] * (2 - len(biases))
    assert len(biases) == 2, "at most two biases"
    _check_shapes(Q, biases)
    if FS.supported(Q) and K.dtype == Q.dtype and V.dtype == Q.dtype:
        return _kernel_path(Q, K, V, biases)
    return _sdpa_path(Q, K, V, biases)


class EvoformerFusedAttention(torch.autograd.Function):
    """Function-style entry kept for API parity (`EvoformerFusedAttention.apply(q, k, v, bias1, bias2)`); autograd
    flows through the fused kernel's own Function."""

    @staticmethod
    def apply(q, k, v, bias1=None, bias2=None):
        return DS4Sci_EvoformerAttention(q, k, v, [bias1, bias2])
