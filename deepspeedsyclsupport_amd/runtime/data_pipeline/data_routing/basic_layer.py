"""Random layerwise token dropping (reference `runtime/data_pipeline/data_routing/basic_layer.py` +
`csrc/random_ltd/{token_sort.cu, gather_scatter.cu}`).

During training each wrapped layer processes only a random subset of `current_seq` tokens per sample (kept in
their original order), the rest bypass it unchanged; at eval every token goes through. Gather / scatter along the
sequence dimension are device index ops (one kernel each), the sorted random subset comes from a single
`topk` over random keys per sample. For contiguous batch-first bf16 device activations they are the gfx950
16-B-vector row gather / scatter kernels (`ops/moe_ops.py` rows_gather / rows_scatter) with their exact adjoints.
"""
import torch
import torch.nn as nn

from ....ops import moe_ops


def _native(x):
    return x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.shape[-1] % 8 == 0


def _flat(idx, S):
    return (idx + S * torch.arange(idx.shape[0], device=idx.device).unsqueeze(1)).reshape(-1)


class _TokenGatherFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, flat):
        ctx.save_for_backward(flat)
        ctx.shape = x.shape
        return moe_ops.rows_gather(x, flat)

    @staticmethod
    def backward(ctx, g):
        (flat, ) = ctx.saved_tensors
        dx = torch.zeros(ctx.shape, dtype=g.dtype, device=g.device)
        moe_ops.rows_scatter(g.contiguous(), flat, dx)  # kept positions are distinct: scatter == scatter-add
        return dx, None


class _TokenScatterFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, full, part, flat):
        ctx.save_for_backward(flat)
        ctx.part_shape = part.shape
        return moe_ops.rows_scatter(part.contiguous(), flat, full.clone())

    @staticmethod
    def backward(ctx, g):
        (flat, ) = ctx.saved_tensors
        g = g.contiguous()
        gpart = moe_ops.rows_gather(g, flat).view(ctx.part_shape)
        gfull = moe_ops.rows_scatter(torch.zeros_like(gpart), flat, g.clone())
        return gfull, gpart, None


def token_sort_(indices, seq_length=None):
    """Sort each row of distinct token positions. Device int32 rows go through the gfx950 bitmap-compaction kernel
    (`moe_kernels.hip` token_sort_kernel, reference `csrc/random_ltd/token_sort.cu`), in place."""
    if indices.is_cuda and seq_length is not None and indices.dtype == torch.int32 and indices.is_contiguous():
        from ....ops.native import hip_ops
        return hip_ops().token_sort_(indices, int(seq_length))
    return torch.sort(indices, dim=-1).values


def mask_gather_gpt(mask, reserved_length):
    """Causal mask of the kept tokens: they keep their relative order, so it is the leading k x k block (reference
    `ops/random_ltd/dropping_utils.py:18-42` gpt_sample_tokens)."""
    return mask[..., :reserved_length, :reserved_length]


def mask_gather_bert(mask, idx):
    """Encoder mask [B, 1, Sq, S] (or [B, 1, 1, S] key-padding) restricted to the kept positions idx [B, k] on both
    the query and the key axis (reference `dropping_utils.py:52-79` bert_sample_tokens / `slice_attn_masks.cu`)."""
    B, k = idx.shape
    if mask.shape[-2] != 1:
        rows = idx.view(B, 1, k, 1).expand(B, mask.shape[1], k, mask.shape[-1])
        mask = torch.gather(mask, 2, rows)
    cols = idx.view(B, 1, 1, k).expand(B, mask.shape[1], mask.shape[2], k)
    return torch.gather(mask, 3, cols)


def token_gather(x, idx, batch_first=True):
    """x [B, S, H] (or [S, B, H]) -> [B, k, H] keeping positions idx [B, k]."""
    if not batch_first:
        x = x.transpose(0, 1)
    out = torch.gather(x, 1, idx.unsqueeze(-1).expand(-1, -1, x.shape[-1]))
    return out if batch_first else out.transpose(0, 1)


def token_scatter_(full, part, idx, batch_first=True):
    """full[b, idx[b, j]] = part[b, j] (in place); returns full."""
    if not batch_first:
        full_v, part_v = full.transpose(0, 1), part.transpose(0, 1)
    else:
        full_v, part_v = full, part
    full_v.scatter_(1, idx.unsqueeze(-1).expand(-1, -1, full_v.shape[-1]), part_v)
    return full


class RandomLayerTokenDrop(nn.Module):

    def __init__(self, layer, batch_first=True):
        super().__init__()
        self.random_ltd_layer = layer
        self.batch_first = batch_first
        self.reserved_length = None
        self.random_ltd_scheduler = None
        self.random_ltd_num_layer = None
        self.random_ltd_initialized = False
        self.mask_name = None
        self.model_type = "decoder"

    def init_config(self, config, scheduler, random_ltd_layer_id):
        self.random_ltd_scheduler = scheduler
        self.random_ltd_layer_id = random_ltd_layer_id
        self.random_ltd_initialized = True
        self.mask_name = config.get("model_mask_name")
        self.model_type = config.get("model_type", "decoder")
        if "hidden_state_order" in config:
            self.batch_first = config["hidden_state_order"] == "batch_seq_dim"

    def forward(self, hidden_states, *args, **kwargs):
        if self.random_ltd_scheduler is not None:
            self.reserved_length = self.random_ltd_scheduler.get_current_seq()
        S = hidden_states.shape[1 if self.batch_first else 0]
        if not self.training or self.reserved_length is None or self.reserved_length >= S:
            return self.random_ltd_layer(hidden_states, *args, **kwargs)
        B = hidden_states.shape[0 if self.batch_first else 1]
        keys = torch.rand(B, S, device=hidden_states.device)
        idx = torch.topk(keys, self.reserved_length, dim=-1).indices
        idx = token_sort_(idx.to(torch.int32), S).long() if idx.is_cuda else token_sort_(idx)
        if self.mask_name is not None and kwargs.get(self.mask_name) is not None:
            m = kwargs[self.mask_name]
            kwargs = dict(kwargs)
            kwargs[self.mask_name] = mask_gather_bert(m, idx) if self.model_type == "encoder" else \
                mask_gather_gpt(m, self.reserved_length)
        native = self.batch_first and _native(hidden_states)
        if native:
            flat = _flat(idx, S)
            part = _TokenGatherFn.apply(hidden_states, flat).view(B, self.reserved_length, -1)
        else:
            part = token_gather(hidden_states, idx, self.batch_first)
        out = self.random_ltd_layer(part, *args, **kwargs)
        rest = out[1:] if isinstance(out, tuple) else None
        out = out[0] if isinstance(out, tuple) else out
        if native and out.dtype == hidden_states.dtype:
            full = _TokenScatterFn.apply(hidden_states, out, flat)
        else:
            full = token_scatter_(hidden_states.clone(), out, idx, self.batch_first)
        return (full, ) + tuple(rest) if rest is not None else full


def convert_to_random_ltd(model, layer_cls):
    """Wrap every instance of `layer_cls` in `model` with RandomLayerTokenDrop (reference helper)."""
    for name, child in list(model.named_children()):
        if isinstance(child, layer_cls):
            setattr(model, name, RandomLayerTokenDrop(child))
        else:
            convert_to_random_ltd(child, layer_cls)
    return model
