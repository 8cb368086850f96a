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
    """Return the kernel-injected replacement for `model` (TP/dtype from the inference `config`). The replacement
    remembers the module it was built from, so `revert_transformer_layer` can hand it back."""
    from .. import comm as dist
    tp = config.tensor_parallel.tp_size if config is not None else 1
    group = config.tensor_parallel.tp_group if config is not None else None
    rank = dist.get_rank(group) if tp > 1 else 0
    dtype = config.dtype if config is not None else torch.bfloat16
    device = next(model.parameters()).device
    injected = convert.from_model(model, group, tp, rank, dtype, device)
    object.__setattr__(injected, "_ds_original_module", model)  # not registered as a submodule
    return injected


@torch.no_grad()
def revert_transformer_layer(orig_layer_impl, model, config=None, preln=False):
    """Inverse of `replace_transformer_layer` (reference `replace_module.py:560-640`, which rebuilds the original
    layers and copies the fused weights back): returns the original module with the injected module's current
    weights written back into it (q/k/v and gate/up un-fused, quantised weights dequantised), so edits made to the
    injected weights survive the round trip. Tensor-parallel injected models are refused: their shards would have to
    be gathered first."""
    orig = getattr(model, "_ds_original_module", None)
    if orig is None:
        raise ValueError("this module was not produced by replace_transformer_layer (no original module attached)")
    if getattr(model, "tp_size", 1) > 1:
        raise NotImplementedError("reverting a tensor-parallel injected model: gather the shards with "
                                  "save_mp_checkpoint_path / state_dict first")
    spec, top, layers = convert.extract(orig)  # views onto the original tensors, in the injected naming
    D, hq, hk = spec.head_dim, spec.num_heads, spec.num_kv_heads

    def back(dst, src):
        if dst is not None and src is not None and dst.numel() == src.numel():
            dst.data.copy_(src.reshape(dst.shape).to(dst.dtype))

    for lw, layer in zip(layers, model.layers):
        qkv = layer._w("qkv_w")
        q, k, v = qkv.split([hq * D, hk * D, hk * D], 0)
        back(lw.get("q_w"), q), back(lw.get("k_w"), k), back(lw.get("v_w"), v)
        if layer.qkv_b is not None and lw.get("q_b") is not None:
            qb, kb, vb = layer.qkv_b.split([hq * D, hk * D, hk * D], 0)
            back(lw["q_b"], qb), back(lw["k_b"], kb), back(lw["v_b"], vb)
        back(lw.get("o_w"), layer._w("o_w")), back(lw.get("o_b"), layer.o_b)
        if not spec.num_experts:
            fc1 = layer._w("fc1_w")
            if "gate_w" in lw:
                g, u = fc1.chunk(2, 0)
                back(lw["gate_w"], g), back(lw["up_w"], u)
            else:
                back(lw.get("fc1_w"), fc1), back(lw.get("fc1_b"), layer.fc1_b)
            back(lw.get("fc2_w"), layer._w("fc2_w")), back(lw.get("fc2_b"), layer.fc2_b)
        for n in ("ln1_w", "ln1_b", "ln2_w", "ln2_b"):
            back(lw.get(n), getattr(layer, n, None))
    back(top.get("embed"), model.embed)
    back(top.get("norm_w"), model.norm_w), back(top.get("norm_b"), model.norm_b)
    if not spec.tie_embeddings:
        back(top.get("lm_head"), model.lm_head[:spec.vocab_size])
    return orig


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
