"""Module-surgery helpers of compression training (reference `compression/helper.py`): attribute paths, swapping
modules for their compression-aware versions, GPT-2 `Conv1D` -> `nn.Linear`, baking one technique in."""
import torch
import torch.nn as nn

from .basic_layer import BNLayer_Compress, Conv2dLayer_Compress, Embedding_Compress, LinearLayer_Compress

COMPRESSIBLE = (nn.Linear, nn.Embedding, nn.Conv2d, nn.BatchNorm2d)


def recursive_getattr(model, module_name):
    for part in module_name.split("."):
        model = getattr(model, part)
    return model


def recursive_setattr(model, module_name, module):
    parent, _, leaf = module_name.rpartition(".")
    setattr(recursive_getattr(model, parent) if parent else model, leaf, module)


def is_module_compressible(module, mpu=None):
    return isinstance(module, COMPRESSIBLE) or type(module).__name__ in ("ColumnParallelLinear", "RowParallelLinear")


def _copy_into(new, old):
    new.load_state_dict(old.state_dict(), strict=False)
    return new


def to_compress_module(m, mpu=None):
    """The compression-aware replacement of `m` (itself when already replaced, None when not compressible)."""
    if isinstance(m, (LinearLayer_Compress, Embedding_Compress, Conv2dLayer_Compress, BNLayer_Compress)):
        return m
    dev, dt = (m.weight.device, m.weight.dtype) if getattr(m, "weight", None) is not None else (None, None)
    if isinstance(m, nn.Linear):
        return _copy_into(LinearLayer_Compress(m.in_features, m.out_features, bias=m.bias is not None, device=dev,
                                               dtype=dt), m)
    if isinstance(m, nn.Embedding):
        return _copy_into(Embedding_Compress(m.num_embeddings, m.embedding_dim, padding_idx=m.padding_idx, device=dev,
                                             dtype=dt), m)
    if isinstance(m, nn.Conv2d):
        return _copy_into(Conv2dLayer_Compress(m.in_channels, m.out_channels, m.kernel_size, stride=m.stride,
                                               padding=m.padding, dilation=m.dilation, groups=m.groups,
                                               bias=m.bias is not None, padding_mode=m.padding_mode, device=dev,
                                               dtype=dt), m)
    if isinstance(m, nn.BatchNorm2d):
        return _copy_into(BNLayer_Compress(m.num_features, eps=m.eps, momentum=m.momentum, affine=m.affine,
                                           track_running_stats=m.track_running_stats, device=dev, dtype=dt), m)
    return None


def module_replacement(model, module_name, compression_technique=None, mpu=None):
    """Swap `model.<module_name>` for its compression-aware version; returns the new module."""
    old = recursive_getattr(model, module_name)
    new = to_compress_module(old, mpu)
    if new is not None and new is not old:
        recursive_setattr(model, module_name, new)
    return new


def compression_preparation(model, compression_technique_list, mpu=None):
    """Replace every compressible module of `model` (reference: done before any technique is enabled)."""
    for name, m in list(model.named_modules()):
        if name and is_module_compressible(m, mpu):
            module_replacement(model, name, mpu=mpu)
    return model


def convert_conv1d_to_linear(model, convert_type):
    """HF GPT-2 style `Conv1D` (weight [in, out], y = x W + b) -> nn.Linear (weight [out, in]) for every module of
    `convert_type` (a class or a class name)."""
    def is_conv1d(m):
        return (isinstance(m, convert_type) if isinstance(convert_type, type) else type(m).__name__ == convert_type)

    for name, m in list(model.named_modules()):
        if name and is_conv1d(m):
            w = m.weight
            lin = nn.Linear(w.shape[0], w.shape[1], bias=getattr(m, "bias", None) is not None, device=w.device,
                            dtype=w.dtype)
            with torch.no_grad():
                lin.weight.copy_(w.t())
                if lin.bias is not None:
                    lin.bias.copy_(m.bias)
            recursive_setattr(model, name, lin)
    return model


@torch.no_grad()
def fix_compression(model, module_name, compression_technique, mask=None, dim_reduction=False):
    """Bake one technique of one module in (reference `helper.py:207`). Returns the kept-index mask for pruning
    techniques (consumers prune their inputs with it)."""
    m = recursive_getattr(model, module_name)
    if compression_technique == "weight_quantization" and hasattr(m, "fix_weight_quantization"):
        m.fix_weight_quantization()
        return None
    if compression_technique == "sparse_pruning" and hasattr(m, "fix_sparse_pruning_helper"):
        m.fix_sparse_pruning_helper()
        return None
    if compression_technique == "row_pruning" and hasattr(m, "fix_row_col_pruning_helper"):
        if mask is not None:
            m.fix_column_pruning(mask) if dim_reduction else m.weight.mul_(mask.view(1, -1).to(m.weight.dtype))
            return mask
        if getattr(m, "row_pruning_enabled", False):
            m.update_masks()
        return m.fix_row_col_pruning_helper(dim_reduction=dim_reduction)
    if compression_technique == "head_pruning" and hasattr(m, "fix_head_pruning_helper"):
        if getattr(m, "head_pruning_enabled", False):
            m.update_masks()
        return m.fix_head_pruning_helper(dim_reduction=dim_reduction)
    if compression_technique == "channel_pruning" and hasattr(m, "fix_channel_pruning_helper"):
        return m.fix_channel_pruning_helper(mask=mask, dim_reduction=dim_reduction)
    return None
