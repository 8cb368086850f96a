"""Kernel-injection entry points (reference `module_inject/replace_module.py:183-640`: replace_transformer_layer,
revert_transformer_layer, generic_injection, ReplaceWithTensorSlicing).

Instead of swapping each HF layer for a fused CUDA module, injection converts the whole decoder into a
`DSInferenceModel` (one implementation parametrised by the architecture spec); see
`inference/model_implementations/convert.py` for the per-architecture policies.
"""
import re

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


class GroupQuantizer:
    """Symmetric group-wise int8 quantiser of weight matrices (reference `replace_module.py:43-83`): returns the
    int8 tensor with a `.scale` attribute holding 1 / step per group, laid out for a tensor-parallel split in
    `count` pieces along `parallel_dim` (each piece gets its own groups, so shards can be cut without
    re-quantising)."""

    def __init__(self, q_int8=True, group_size=1, num_bits=8, num_groups=0):
        self.group_size = group_size
        self.num_bits = num_bits
        self.q_int8 = q_int8
        self.num_groups = num_groups

    def quantize(self, inputs, qkv=True, count=1, parallel_dim=0):
        if not self.q_int8 or not qkv:
            inputs = torch.nn.Parameter(inputs, requires_grad=False)
            inputs.scale = torch.empty(1)
            return inputs
        q_range = 2**self.num_bits
        num_groups = self.num_groups if self.num_groups > 0 else inputs.shape[0] // self.group_size
        x = inputs.to(torch.float32)
        grouped = x.reshape(num_groups, -1)
        step = (2 * grouped.abs().amax(dim=1, keepdim=True)).clamp_min(1e-12) / q_range
        q = (grouped / step).round().clamp(-q_range // 2, q_range // 2 - 1).to(torch.int8).reshape(inputs.shape)
        out = torch.nn.Parameter(q, requires_grad=False)
        # per-piece scales: quantise each tensor-parallel piece by its own groups, stacked piece-major
        scales = []
        for piece in x.chunk(max(count, 1), dim=parallel_dim):
            g = piece.reshape(num_groups, -1) if piece.numel() % num_groups == 0 else piece.reshape(1, -1)
            scales.append((q_range / (2 * g.abs().amax(dim=1)).clamp_min(1e-12)))
        out.scale = torch.cat([s.reshape(-1) for s in scales]).unsqueeze(0)
        return out


def get_transformer_name(replaced_module):
    """Qualified name of the ModuleList that holds the model's transformer layers."""
    best = ""
    for name, child in replaced_module.named_modules():
        if isinstance(child, torch.nn.ModuleList) and len(child) > 0 and \
                sum(1 for _ in child[0].modules()) > 2 and (not best or len(child) >= 1):
            best = best or name
    return best


def skip_level_0_prefix(model, state_dict):
    """Models whose checkpoints carry no top-level prefix (BLOOM / OPT style) are loaded from level 1 down."""
    key = re.search(r": (.*?)Model", str(type(model)))
    if key is None:
        key = re.search(r": (.*?)Stack", str(type(model)))
    if key is None:
        key = re.match(r"(.*?)Model", type(model).__name__)
    return key is not None and key.group(1).split(".")[-1].lower() in ("bloom", "opt")


def replace_module(model, orig_class, replace_fn, _replace_policy=None, checkpoint=None):
    """Swap every instance of `orig_class` (a class, or None to use each policy's `_orig_layer_class`) for
    `replace_fn(child, policy_class, layer_id)` (reference `replace_module.py:586-627`). `_replace_policy` narrows the
    policies tried to one class. Returns the model."""
    from .containers import replace_policies
    policies = [_replace_policy] if _replace_policy is not None else list(replace_policies)
    targets = {}
    if orig_class is not None:
        targets[orig_class] = policies[0] if _replace_policy is not None else None
    else:
        for pol in policies:
            cls = getattr(pol, "_orig_layer_class", None)  # (set by the policy the first time it is constructed)
            for c in (cls if isinstance(cls, (list, tuple)) else [cls]):
                if c is not None:
                    targets[c] = pol
    layer_id = 0
    for name, child in list(model.named_modules()):
        if not name:
            continue
        pol = next((p for c, p in targets.items() if isinstance(child, c)), "none")
        if pol == "none":
            continue
        new = replace_fn(child, pol, layer_id)
        parent_name, _, leaf = name.rpartition(".")
        parent = model.get_submodule(parent_name) if parent_name else model
        setattr(parent, leaf, new)
        layer_id += 1
    return model

