"""DS4Science Evoformer attention (reference `ops/deepspeed4science/evoformer_attn.py:59-106`):
out = softmax(Q K^T / sqrt(D) + bias1 + bias2) V over [B, N, S, H, D] tensors (MSA row/column attention in
AlphaFold-style models), bias1 = per-key mask bias [B, N, 1, 1, S], bias2 = pair bias [B, 1, H, S, S]; gradients
flow to Q, K, V and both biases. Runs on the fused SDPA kernels with the summed bias (B*N folded into batch)."""
import math

import torch
import torch.nn.functional as F


def DS4Sci_EvoformerAttention(Q, K, V, biases):
    assert Q.dim() == 5, "expected [B, N, S, H, D]"
    B, N, S, H, D = Q.shape
    biases = list(biases) + [None] * (2 - len(biases))
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


class EvoformerFusedAttention(torch.autograd.Function):
    """Function-style entry kept for API parity; autograd flows through the SDPA path above."""

    @staticmethod
    def apply(q, k, v, bias1=None, bias2=None):
        return DS4Sci_EvoformerAttention(q, k, v, [bias1, bias2])
