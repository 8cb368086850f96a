"""Random-LTD token sampling / gather / scatter (reference `ops/random_ltd/dropping_utils.py`).

Sampling draws `reserved_length` distinct positions per (layer, sample) with one `topk` over random keys and sorts
them (kept tokens stay in order); gather / scatter are the gfx950 row kernels for batch-first bf16 device
activations (`ops/moe_ops.py`) and index ops otherwise. The autograd functions keep the reference's calling
convention: GatherTokens returns (activations, gathered), ScatterTokens returns the scattered full tensor."""
import torch

from ...runtime.data_pipeline.data_routing.basic_layer import (_flat, _native, mask_gather_bert, mask_gather_gpt,
                                                                token_gather, token_scatter_, token_sort_)
from .. import moe_ops


def _sample(reserved_length, seq_length, batch_size, layers, device):
    keys = torch.rand(layers * batch_size, seq_length, device=device)
    idx = torch.topk(keys, reserved_length, dim=-1).indices.to(torch.int32)
    idx = token_sort_(idx.contiguous(), seq_length)
    return idx.reshape(layers, batch_size, reserved_length)


def gpt_sample_tokens(reserved_length, seq_length, batch_size, layers=1, device="cpu", attn_mask=None):
    """-> (indices [layers, B, k] int32 sorted, causal mask [B, 1, k, k] or None)."""
    idx = _sample(reserved_length, seq_length, batch_size, layers, device)
    return idx, (mask_gather_gpt(attn_mask, reserved_length) if attn_mask is not None else None)


def bert_sample_tokens(reserved_length, seq_length, batch_size, layers=1, device="cpu", attn_mask=None):
    """-> (indices [layers, B, k], per-layer encoder masks [layers][B, 1, k, k] gathered at the kept positions)."""
    assert attn_mask is not None, "bert_sample_tokens needs the attention mask"
    idx = _sample(reserved_length, seq_length, batch_size, layers, device)
    masks = [mask_gather_bert(attn_mask, idx[l].long()) for l in range(layers)]
    return idx, masks


def _gather(x, idx, batch_first):
    if batch_first and _native(x):
        B, S = x.shape[0], x.shape[1]
        return moe_ops.rows_gather(x, _flat(idx.long(), S)).view(B, idx.shape[1], -1)
    return token_gather(x, idx.long(), batch_first)


def _scatter(full, part, idx, batch_first):
    if batch_first and _native(full) and part.dtype == full.dtype:
        S = full.shape[1]
        return moe_ops.rows_scatter(part.contiguous(), _flat(idx.long(), S), full)
    return token_scatter_(full, part, idx.long(), batch_first)


class GatherTokens(torch.autograd.Function):

    @staticmethod
    def forward(ctx, activations, sorted_indices, batch_first):
        ctx.save_for_backward(sorted_indices)
        ctx.batch_first = batch_first
        return activations, _gather(activations, sorted_indices, batch_first)

    @staticmethod
    def backward(ctx, a_grad, g_grad):
        (idx, ) = ctx.saved_tensors
        return _scatter(a_grad.clone(), g_grad.contiguous(), idx, ctx.batch_first), None, None


class ScatterTokens(torch.autograd.Function):

    @staticmethod
    def forward(ctx, all_activations, layer_activations, sorted_indices, batch_first):
        ctx.save_for_backward(sorted_indices)
        ctx.batch_first = batch_first
        return _scatter(all_activations.clone(), layer_activations, sorted_indices, batch_first)

    @staticmethod
    def backward(ctx, out_grad):
        (idx, ) = ctx.saved_tensors
        out_grad = out_grad.contiguous()
        return out_grad, _gather(out_grad, idx, ctx.batch_first), None, None
