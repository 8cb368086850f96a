"""Compression-aware layers (reference `compression/basic_layer.py:17-840`): weight quantization (QAT with
straight-through estimator and bit-width annealing down to ternary / binary), activation quantization,
unstructured (sparse), row, head and channel pruning — `l1` masks from weight magnitudes, or `topk` masks from
learnable scores trained through `TopKBinarizer` — applied in forward; `fix_*` helpers bake them in. Also the
Conv2d / BatchNorm2d layers used by channel pruning and the tensor-parallel linear variants.

Fake quantisation of 4/8-bit device tensors runs on the gfx950 group-quantize + dequantize kernels.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class _STEQuant(torch.autograd.Function):
    """fake-quantise in forward, identity gradient (straight-through)."""

    @staticmethod
    def forward(ctx, w, bits, groups, symmetric, stochastic):
        return fake_quant(w, bits, groups, symmetric, stochastic)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None, None


def fake_quant(w, bits, groups=1, symmetric=True, stochastic=False):
    if bits >= 16:
        return w
    if bits <= 2:  # ternary / binary weights (compression/utils.py)
        from .utils import quantizer_for
        return quantizer_for(bits).apply(w.detach(), bits, None, None, groups)
    n = w.numel()
    groups = max(1, min(groups, n))
    while n % groups:
        groups -= 1
    gs = n // groups
    if w.is_cuda and bits in (4, 8) and w.dtype in (torch.float32, torch.bfloat16, torch.float16):
        from ..ops.quantizer import dequantize, quantize
        qt = quantize(w.detach().contiguous(), group_size=gs, bits=bits, symmetric=symmetric,
                      stochastic_rounding=stochastic)
        return dequantize(qt, w.dtype).view_as(w)
    x = w.detach().float().reshape(groups, gs)
    if symmetric:
        qmax = 2**(bits - 1) - 1
        scale = x.abs().amax(1, keepdim=True).clamp_min(1e-12) / qmax
        t = x / scale
        t = torch.floor(t + torch.rand_like(t)) if stochastic else torch.round(t)
        q = t.clamp(-qmax, qmax) * scale
    else:
        lo, hi = x.amin(1, keepdim=True), x.amax(1, keepdim=True)
        scale = (hi - lo).clamp_min(1e-12) / (2**bits - 1)
        t = (x - lo) / scale
        t = torch.floor(t + torch.rand_like(t)) if stochastic else torch.round(t)
        q = t.clamp(0, 2**bits - 1) * scale + lo
    return q.reshape(w.shape).to(w.dtype)


class QuantAct(nn.Module):
    """Activation fake-quantisation with dynamic (per batch) or static (EMA-calibrated) range."""

    def __init__(self, act_range_momentum=0.95, quant_mode="symmetric", bits=8, range_calibration="dynamic"):
        super().__init__()
        self.momentum = act_range_momentum
        self.symmetric = quant_mode == "symmetric"
        self.bits = bits
        self.static = range_calibration == "static"
        self.register_buffer("x_min_max", torch.zeros(2))

    def forward(self, x):
        if self.static:
            if self.training:
                mn, mx = x.detach().min(), x.detach().max()
                if self.x_min_max.abs().sum() == 0:
                    self.x_min_max.copy_(torch.stack([mn, mx]))
                else:
                    self.x_min_max.mul_(self.momentum).add_(torch.stack([mn, mx]) * (1 - self.momentum))
            lo, hi = self.x_min_max[0], self.x_min_max[1]
        else:
            lo, hi = x.detach().min(), x.detach().max()
        if self.symmetric:
            qmax = 2**(self.bits - 1) - 1
            scale = torch.maximum(lo.abs(), hi.abs()).clamp_min(1e-12) / qmax
            q = torch.round(x / scale).clamp(-qmax, qmax) * scale
        else:
            scale = (hi - lo).clamp_min(1e-12) / (2**self.bits - 1)
            q = torch.round((x - lo) / scale).clamp(0, 2**self.bits - 1) * scale + lo
        return x + (q - x).detach()


def _topk_mask(scores, dense_ratio):
    k = max(1, int(math.ceil(scores.numel() * dense_ratio)))
    thr = torch.topk(scores.reshape(-1), k).values[-1]
    return (scores >= thr).to(scores.dtype)


class LinearLayer_Compress(nn.Linear):

    def __init__(self, *args, bias=True, **kwargs):
        super().__init__(*args, bias=bias, **kwargs)
        self.weight_quantization_enabled = False
        self.weight_quantization_enabled_in_forward = False
        self.sparse_pruning_enabled = False
        self.row_pruning_enabled = False
        self.head_pruning_enabled = False
        self.activation_quantization_enabled = False
        self.activation_quantization_method = None
        self.sparse_pruning_method = None
        self.row_pruning_method = None
        self.head_pruning_method = None
        self._step = 0

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}, "
                f"wq={self.weight_quantization_enabled}, sparse={self.sparse_pruning_enabled}, "
                f"row={self.row_pruning_enabled}, head={self.head_pruning_enabled}, "
                f"aq={self.activation_quantization_enabled}")

    # ------------------------------------------------------------------------------------------ enable
    def enable_weight_quantization(self, start_bits, target_bits, quantization_period,
                                   weight_quantization_enabled_in_forward, quantization_type, num_groups):
        self.weight_quantization_enabled = True
        self.weight_quantization_enabled_in_forward = weight_quantization_enabled_in_forward
        self.wq_start_bits, self.wq_target_bits = int(start_bits), int(target_bits)
        self.wq_period = max(int(quantization_period), 1)
        self.wq_symmetric = quantization_type == "symmetric"
        self.wq_groups = int(num_groups)
        self.wq_bits = self.wq_start_bits
        if not weight_quantization_enabled_in_forward:
            # per-weight MoQ schedule consumed by runtime/quantize.py after each optimizer step (reference
            # `compression/basic_layer.py:79-84`)
            self.weight.start_bits = self.wq_start_bits
            self.weight.target_bits = self.wq_target_bits
            self.weight.q_period = self.wq_period

    def enable_activation_quantization(self, bits, quantization_type, range_calibration):
        self.activation_quantization_enabled = True
        self.activation_quantizer = QuantAct(quant_mode=quantization_type, bits=bits,
                                             range_calibration=range_calibration)

    def enable_sparse_pruning(self, ratio, method):
        self.sparse_pruning_enabled = True
        self.sparse_pruning_ratio = ratio
        self.sparse_pruning_method = method
        self.register_buffer("sparse_pruning_mask", torch.ones_like(self.weight))
        if method == "topk":  # learnable importance scores (movement pruning), initialised from |w|
            self.sparse_mask_scores = nn.Parameter(self.weight.detach().abs().clone())

    def enable_row_pruning(self, ratio, method):
        self.row_pruning_enabled = True
        self.row_pruning_ratio = ratio
        self.row_pruning_method = method
        self.register_buffer("row_pruning_mask", torch.ones(self.out_features, 1, device=self.weight.device,
                                                            dtype=self.weight.dtype))

    def enable_head_pruning(self, ratio, method, num_heads):
        self.head_pruning_enabled = True
        self.head_pruning_ratio = ratio
        self.head_pruning_method = method
        self.num_heads = num_heads
        self.register_buffer("head_pruning_mask", torch.ones(1, num_heads, device=self.weight.device,
                                                             dtype=self.weight.dtype))

    # ------------------------------------------------------------------------------------------ masks
    def _sparse_mask(self):
        if self.sparse_pruning_method == "topk":
            from .utils import TopKBinarizer
            return TopKBinarizer.apply(self.sparse_mask_scores, self.sparse_pruning_ratio, False)
        return self.sparse_pruning_mask

    @torch.no_grad()
    def update_masks(self):
        w = self.weight.detach().float()
        if self.sparse_pruning_enabled:
            scores = self.sparse_mask_scores.detach() if self.sparse_pruning_method == "topk" else w.abs()
            self.sparse_pruning_mask.copy_(_topk_mask(scores, self.sparse_pruning_ratio))
        if self.row_pruning_enabled:
            self.row_pruning_mask.copy_(_topk_mask(w.abs().sum(1), self.row_pruning_ratio).view(-1, 1))
        if self.head_pruning_enabled:
            # o-projection style: columns are grouped per head
            hs = self.in_features // self.num_heads
            scores = w.abs().view(self.out_features, self.num_heads, hs).sum((0, 2))
            self.head_pruning_mask.copy_(_topk_mask(scores, self.head_pruning_ratio).view(1, -1))

    def _bit_schedule(self):
        # anneal from start_bits to target_bits, one bit per `quantization_period` steps
        if self.wq_bits > self.wq_target_bits and self._step > 0 and self._step % self.wq_period == 0:
            self.wq_bits -= 1

    def effective_weight(self):
        w = self.weight
        if self.sparse_pruning_enabled:
            w = w * self._sparse_mask()
        if self.row_pruning_enabled:
            w = w * self.row_pruning_mask
        if self.head_pruning_enabled:
            hs = self.in_features // self.num_heads
            w = w * self.head_pruning_mask.repeat_interleave(hs, 1)
        if self.weight_quantization_enabled and self.weight_quantization_enabled_in_forward:
            w = _STEQuant.apply(w, self.wq_bits, self.wq_groups, self.wq_symmetric, False)
        return w

    def forward(self, x, skip_bias_add=False):
        if self.training:
            self._step += 1
            if self.weight_quantization_enabled:
                self._bit_schedule()
        if self.activation_quantization_enabled:
            x = self.activation_quantizer(x)
        w = self.effective_weight()
        b = self.bias
        if b is not None and self.row_pruning_enabled:
            b = b * self.row_pruning_mask.view(-1)
        if skip_bias_add:
            return F.linear(x, w), b
        return F.linear(x, w, b)

    # ------------------------------------------------------------------------------------------ fix (bake in)
    @torch.no_grad()
    def fix_weight_quantization(self):
        if self.weight_quantization_enabled:
            self.weight.copy_(fake_quant(self.weight, self.wq_target_bits, self.wq_groups, self.wq_symmetric))
            self.weight_quantization_enabled = False

    @torch.no_grad()
    def fix_sparse_pruning_helper(self):
        if self.sparse_pruning_enabled:
            self.update_masks()
            self.weight.mul_(self.sparse_pruning_mask)
            self.sparse_pruning_enabled = False
            del self.sparse_pruning_mask
            if hasattr(self, "sparse_mask_scores"):
                del self.sparse_mask_scores

    @torch.no_grad()
    def fix_row_col_pruning_helper(self, mask=None, dim_reduction=False):
        """Physically drop pruned output rows (returns the kept-row mask for the consumer's columns)."""
        if mask is None and not self.row_pruning_enabled:
            return None
        keep = (mask if mask is not None else self.row_pruning_mask.view(-1)).bool()
        if dim_reduction:
            self.weight = nn.Parameter(self.weight[keep].clone())
            if self.bias is not None:
                self.bias = nn.Parameter(self.bias[keep].clone())
            self.out_features = int(keep.sum())
        else:
            self.weight.mul_(keep.view(-1, 1).to(self.weight.dtype))
            if self.bias is not None:
                self.bias.mul_(keep.to(self.bias.dtype))
        if self.row_pruning_enabled:
            self.row_pruning_enabled = False
            del self.row_pruning_mask
        return keep

    @torch.no_grad()
    def fix_column_pruning(self, keep):
        """Drop input columns whose producer rows were pruned."""
        self.weight = nn.Parameter(self.weight[:, keep].clone())
        self.in_features = int(keep.sum())

    @torch.no_grad()
    def fix_head_pruning_helper(self, dim_reduction=False):
        if not self.head_pruning_enabled:
            return None
        hs = self.in_features // self.num_heads
        keep = self.head_pruning_mask.view(-1).bool().repeat_interleave(hs)
        if dim_reduction:
            self.weight = nn.Parameter(self.weight[:, keep].clone())
            self.in_features = int(keep.sum())
        else:
            self.weight.mul_(keep.view(1, -1).to(self.weight.dtype))
        self.head_pruning_enabled = False
        del self.head_pruning_mask
        return keep


class Embedding_Compress(nn.Embedding):

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.weight_quantization_enabled = False

    def enable_weight_quantization(self, start_bits, target_bits, quantization_period,
                                   weight_quantization_enabled_in_forward, quantization_type, num_groups):
        self.weight_quantization_enabled = True
        self.wq_target_bits = int(target_bits)
        self.wq_groups = int(num_groups)
        self.wq_symmetric = quantization_type == "symmetric"

    def forward(self, x):
        w = self.weight
        if self.weight_quantization_enabled:
            w = _STEQuant.apply(w, self.wq_target_bits, self.wq_groups, self.wq_symmetric, False)
        return F.embedding(x, w, self.padding_idx, self.max_norm, self.norm_type, self.scale_grad_by_freq,
                           self.sparse)

    @torch.no_grad()
    def fix_weight_quantization(self):
        if self.weight_quantization_enabled:
            self.weight.copy_(fake_quant(self.weight, self.wq_target_bits, self.wq_groups, self.wq_symmetric))
            self.weight_quantization_enabled = False


class Conv2dLayer_Compress(nn.Conv2d):
    """Conv2d with weight quantization and output-channel pruning (reference `basic_layer.py:404`)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.weight_quantization_enabled = False
        self.channel_pruning_enabled = False
        self.activation_quantization_enabled = False

    def enable_weight_quantization(self, start_bits, target_bits, quantization_period,
                                   weight_quantization_enabled_in_forward, quantization_type, num_groups):
        self.weight_quantization_enabled = True
        self.wq_target_bits = int(target_bits)
        self.wq_groups = int(num_groups)
        self.wq_symmetric = quantization_type == "symmetric"

    def enable_activation_quantization(self, bits, quantization_type, range_calibration):
        self.activation_quantization_enabled = True
        self.activation_quantizer = QuantAct(quant_mode=quantization_type, bits=bits,
                                             range_calibration=range_calibration)

    def enable_channel_pruning(self, ratio, method):
        self.channel_pruning_enabled = True
        self.channel_pruning_ratio = ratio
        self.channel_pruning_method = method
        self.register_buffer("channel_pruning_mask", torch.ones(self.out_channels, 1, 1, 1, device=self.weight.device,
                                                                dtype=self.weight.dtype))
        if method == "topk":
            self.channel_mask_scores = nn.Parameter(
                self.weight.detach().abs().sum((1, 2, 3)).view(-1, 1, 1, 1).clone())

    def _channel_mask(self):
        if self.channel_pruning_method == "topk":
            from .utils import TopKBinarizer
            return TopKBinarizer.apply(self.channel_mask_scores, self.channel_pruning_ratio, False)
        return self.channel_pruning_mask

    @torch.no_grad()
    def update_masks(self):
        if self.channel_pruning_enabled:
            scores = (self.channel_mask_scores.detach().view(-1) if self.channel_pruning_method == "topk"
                      else self.weight.detach().float().abs().sum((1, 2, 3)))
            self.channel_pruning_mask.copy_(_topk_mask(scores, self.channel_pruning_ratio).view(-1, 1, 1, 1))

    def forward(self, x):
        if self.activation_quantization_enabled:
            x = self.activation_quantizer(x)
        w, b = self.weight, self.bias
        if self.channel_pruning_enabled:
            m = self._channel_mask()
            w = w * m
            if b is not None:
                b = b * m.view(-1)
        if self.weight_quantization_enabled:
            w = _STEQuant.apply(w, self.wq_target_bits, self.wq_groups, self.wq_symmetric, False)
        return self._conv_forward(x, w, b)

    @torch.no_grad()
    def fix_weight_quantization(self):
        if self.weight_quantization_enabled:
            self.weight.copy_(fake_quant(self.weight, self.wq_target_bits, self.wq_groups, self.wq_symmetric))
            self.weight_quantization_enabled = False

    @torch.no_grad()
    def fix_channel_pruning_helper(self, mask=None, dim_reduction=False):
        """Output channels kept (bool [out]); with dim_reduction the pruned channels are physically removed.
        `mask` given: prune INPUT channels instead (this conv consumes a pruned producer)."""
        if mask is not None:
            keep = mask.bool()
            if dim_reduction:
                self.weight = nn.Parameter(self.weight[:, keep].clone())
                self.in_channels = int(keep.sum())
            else:
                self.weight.mul_(keep.view(1, -1, 1, 1).to(self.weight.dtype))
            return keep
        if not self.channel_pruning_enabled:
            return None
        self.update_masks()
        keep = self.channel_pruning_mask.view(-1).bool()
        if dim_reduction:
            self.weight = nn.Parameter(self.weight[keep].clone())
            if self.bias is not None:
                self.bias = nn.Parameter(self.bias[keep].clone())
            self.out_channels = int(keep.sum())
        else:
            self.weight.mul_(keep.view(-1, 1, 1, 1).to(self.weight.dtype))
            if self.bias is not None:
                self.bias.mul_(keep.to(self.bias.dtype))
        self.channel_pruning_enabled = False
        del self.channel_pruning_mask
        if hasattr(self, "channel_mask_scores"):
            del self.channel_mask_scores
        return keep


class BNLayer_Compress(nn.BatchNorm2d):
    """BatchNorm2d that follows a channel-pruned conv (reference `basic_layer.py:611`)."""

    @torch.no_grad()
    def fix_channel_pruning_helper(self, mask, dim_reduction=False):
        keep = mask.bool()
        if dim_reduction:
            self.weight = nn.Parameter(self.weight[keep].clone())
            self.bias = nn.Parameter(self.bias[keep].clone())
            self.running_mean = self.running_mean[keep].clone()
            self.running_var = self.running_var[keep].clone()
            self.num_features = int(keep.sum())
        else:
            self.weight.mul_(keep.to(self.weight.dtype))
            self.bias.mul_(keep.to(self.bias.dtype))
        return keep


# ------------------------------------------------------------------------------------------ tensor-parallel variants
class _MPRegion(torch.autograd.Function):
    """fwd/bwd pairs of the model-parallel region ops: 'copy' (identity / all-reduce), 'reduce' (all-reduce /
    identity), 'gather' (all-gather last dim / split)."""

    @staticmethod
    def forward(ctx, x, kind, group):
        import torch.distributed as dist
        ctx.kind, ctx.group = kind, group
        ws = dist.get_world_size(group)
        if ws == 1 or kind == "copy":
            return x
        if kind == "reduce":
            y = x.clone()
            dist.all_reduce(y, group=group)
            return y
        parts = [torch.empty_like(x) for _ in range(ws)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):
        import torch.distributed as dist
        ws = dist.get_world_size(ctx.group)
        if ws == 1 or ctx.kind == "reduce":
            return g, None, None
        if ctx.kind == "copy":
            g = g.clone()
            dist.all_reduce(g, group=ctx.group)
            return g, None, None
        return g.chunk(ws, dim=-1)[dist.get_rank(ctx.group)].contiguous(), None, None


class ColumnParallelLinear_Compress(LinearLayer_Compress):
    """Output-dim sharded compression linear (reference `basic_layer.py:767`): y_local = x W_local^T, optionally
    gathered over the model-parallel group."""

    def __init__(self, mpu, input_size, output_size, bias=True, gather_output=True, skip_bias_add=False, **kw):
        self.mp_group = mpu.get_model_parallel_group()
        ws = mpu.get_model_parallel_world_size()
        assert output_size % ws == 0, "output size must divide the model-parallel size"
        super().__init__(input_size, output_size // ws, bias=bias, **kw)
        self.gather_output, self.skip_bias = gather_output, skip_bias_add

    def forward(self, x):
        x = _MPRegion.apply(x, "copy", self.mp_group)
        if self.skip_bias:
            y, b = super().forward(x, skip_bias_add=True)
        else:
            y, b = super().forward(x), None
        if self.gather_output:
            y = _MPRegion.apply(y, "gather", self.mp_group)
        return (y, b) if self.skip_bias else y


class RowParallelLinear_Compress(LinearLayer_Compress):
    """Input-dim sharded compression linear (reference `basic_layer.py:802`): partial products all-reduced over the
    model-parallel group, bias added once after the reduction."""

    def __init__(self, mpu, input_size, output_size, bias=True, input_is_parallel=True, skip_bias_add=False, **kw):
        self.mp_group = mpu.get_model_parallel_group()
        ws = mpu.get_model_parallel_world_size()
        self.mp_rank = mpu.get_model_parallel_rank()
        self.mp_ws = ws
        assert input_size % ws == 0, "input size must divide the model-parallel size"
        super().__init__(input_size // ws, output_size, bias=bias, **kw)
        self.input_is_parallel, self.skip_bias = input_is_parallel, skip_bias_add

    def forward(self, x):
        if not self.input_is_parallel:
            x = x.chunk(self.mp_ws, dim=-1)[self.mp_rank]
        y, b = super().forward(x, skip_bias_add=True)
        y = _MPRegion.apply(y, "reduce", self.mp_group)
        if self.skip_bias:
            return y, b
        return y + b if b is not None else y
