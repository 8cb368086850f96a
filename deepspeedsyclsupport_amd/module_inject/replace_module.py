"""Kernel-injection entry points (reference `module_inject/replace_module.py:183-640`: replace_transformer_layer,
revert_transformer_layer, generic_injection, ReplaceWithTensorSlicing).

Instead of swapping each HF layer for a fused CUDA module, injection converts the whole decoder into a
`DSInferenceModel` (one implementation parametrised by the architecture spec); see
`inference/model_implementations/convert.py` for the per-architecture policies.
"""
import torch

from ..inference.model_implementations import convert


class ReplaceWithTensorSlicing:
    """Copy a full tensor into a TP shard (reference replace_module.py:33-180), row (dim 0) or column (dim 1)."""

    def __init__(self, mp_group=None, mp_size=1, out_dim=1, in_dim=0):
        from .. import comm as dist
        self.gpu_index = dist.get_rank(group=mp_group) if mp_group is not None else 0
        self.mp_size = mp_size
        self.out_dim, self.in_dim = out_dim, in_dim

    def copy(self, dst, src, int8=False, allocate_tensor=False):
        if src is None:
            return src
        if dst.shape == src.shape:
            dst.data.copy_(src)
            return dst
        dim = 0 if dst.shape[0] != src.shape[0] else 1
        n = src.shape[dim] // self.mp_size
        dst.data.copy_(src.narrow(dim, self.gpu_index * n, n))
        return dst

    def qkv_copy(self, dst, src, int8=False, allocate_tensor=False):
        """Fused [q|k|v] stacked along dim 0: take this rank's slice of each part."""
        parts = src.chunk(3, 0)
        n = parts[0].shape[0] // self.mp_size
        dst.data.copy_(torch.cat([p[self.gpu_index * n:(self.gpu_index + 1) * n] for p in parts], 0))
        return dst


def replace_transformer_layer(orig_layer_impl, model, checkpoint_dict=None, config=None, model_config=None):
    """Return the kernel-injected replacement for `model` (TP/dtype from the inference `config`)."""
    from .. import comm as dist
    tp = config.tensor_parallel.tp_size if config is not None else 1
    group = config.tensor_parallel.tp_group if config is not None else None
    rank = dist.get_rank(group) if tp > 1 else 0
    dtype = config.dtype if config is not None else torch.bfloat16
    device = next(model.parameters()).device
    return convert.from_model(model, group, tp, rank, dtype, device)


def revert_transformer_layer(orig_layer_impl, model, config, preln=False):
    raise NotImplementedError("kernel injection builds a new module; keep a reference to the original model instead")


def generic_injection(module, dtype=None, enable_cuda_graph=True):
    """Diffusers pipeline injection (reference `replace_module.py:generic_injection`): for a pipeline object, the
    UNet / VAE attention modules and transformer blocks are replaced by the fused MI355X modules and the UNet / VAE /
    text encoder are wrapped in HIP-graph replaying wrappers (`module_inject/diffusers.py`). A plain `nn.Module` is
    returned unchanged (as in the reference, which only injects pipelines here)."""
    if isinstance(module, torch.nn.Module):
        return module
    from .diffusers import inject_pipeline
    inject_pipeline(module, dtype=dtype, enable_cuda_graph=enable_cuda_graph)
    return module
