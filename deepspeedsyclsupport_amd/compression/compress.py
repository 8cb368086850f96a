"""Compression entry points (reference `compression/compress.py:100-240`, `compression/scheduler.py`,
`compression/helper.py`): `init_compression` swaps matching nn.Linear / nn.Embedding modules for their
compression-aware versions and enables the configured techniques; `compression_scheduler` turns techniques on at
their `schedule_offset`; `redundancy_clean` bakes masks / quantisation in (and, for row pruning, shrinks the layers
and the consumers named in `related_modules`).

Config (same keys as the reference):
  "compression_training": {
    "weight_quantization": {"shared_parameters": {...}, "different_groups": {"g": {"params": {...}, "modules": [...]}}},
    "activation_quantization": {...}, "sparse_pruning": {...}, "row_pruning": {...}, "head_pruning": {...},
    "layer_reduction": {"enabled": ..., "keep_number_layer": k, "module_name_prefix": "...", "teacher_layer": [...]}}
"""
import fnmatch
import json
import re

import torch
import torch.nn as nn

from .basic_layer import Embedding_Compress, LinearLayer_Compress

TECHNIQUES = ("weight_quantization", "activation_quantization", "sparse_pruning", "row_pruning", "head_pruning",
              "channel_pruning")


def _cfg(deepspeed_config):
    if isinstance(deepspeed_config, str):
        with open(deepspeed_config) as f:
            deepspeed_config = json.load(f)
    if hasattr(deepspeed_config, "_param_dict"):
        deepspeed_config = deepspeed_config._param_dict
    return deepspeed_config.get("compression_training", {})


def _match(name, patterns):
    for p in patterns:
        if p == "*" or fnmatch.fnmatch(name, p) or p in name:
            return True
        try:
            if re.fullmatch(p, name):
                return True
        except re.error:
            pass
    return False


def recursive_getattr(model, name):
    for part in name.split("."):
        model = getattr(model, part)
    return model


def recursive_setattr(model, name, module):
    parent, _, leaf = name.rpartition(".")
    setattr(recursive_getattr(model, parent) if parent else model, leaf, module)


def _to_compress(m):
    if isinstance(m, (LinearLayer_Compress, Embedding_Compress)):
        return m
    if isinstance(m, nn.Linear):
        new = LinearLayer_Compress(m.in_features, m.out_features, bias=m.bias is not None, device=m.weight.device,
                                   dtype=m.weight.dtype)
    elif isinstance(m, nn.Embedding):
        new = Embedding_Compress(m.num_embeddings, m.embedding_dim, padding_idx=m.padding_idx,
                                 device=m.weight.device, dtype=m.weight.dtype)
    else:
        return None
    new.load_state_dict(m.state_dict(), strict=False)
    return new


def _groups(tech_cfg):
    shared = tech_cfg.get("shared_parameters", {})
    for gname, g in tech_cfg.get("different_groups", {}).items():
        yield gname, shared, g.get("params", {}), g.get("modules", ["*"]), g.get("related_modules")


def _enable(m, tech, shared, params):
    if tech == "weight_quantization":
        m.enable_weight_quantization(params.get("start_bits", 8), params.get("target_bits", 8),
                                     params.get("quantization_period", 1),
                                     shared.get("quantize_weight_in_forward", True),
                                     shared.get("quantization_type", "symmetric"), shared.get("quantize_groups", 1))
    elif tech == "activation_quantization" and isinstance(m, LinearLayer_Compress):
        m.enable_activation_quantization(params.get("bits", 8), shared.get("quantization_type", "symmetric"),
                                         shared.get("range_calibration", "dynamic"))
    elif tech == "sparse_pruning" and isinstance(m, LinearLayer_Compress):
        m.enable_sparse_pruning(params.get("dense_ratio", 0.5), shared.get("method", "l1"))
    elif tech == "row_pruning" and isinstance(m, LinearLayer_Compress):
        m.enable_row_pruning(params.get("dense_ratio", 0.5), shared.get("method", "l1"))
    elif tech == "head_pruning" and isinstance(m, LinearLayer_Compress):
        m.enable_head_pruning(params.get("dense_ratio", 0.5), shared.get("method", "topk"),
                              shared.get("num_heads", 1))


def _layer_reduction(model, lr):
    if not lr.get("enabled", False):
        return
    prefix = lr["module_name_prefix"]
    keep = lr.get("teacher_layer", list(range(lr["keep_number_layer"])))
    layers = recursive_getattr(model, prefix)
    recursive_setattr(model, prefix, nn.ModuleList([layers[i] for i in keep]))


def init_compression(model, deepspeed_config, teacher_model=None, mpu=None):
    cc = _cfg(deepspeed_config)
    target = model.module if hasattr(model, "module") and isinstance(model.module, nn.Module) else model
    _layer_reduction(target, cc.get("layer_reduction", {}))
    names = [n for n, m in target.named_modules() if isinstance(m, (nn.Linear, nn.Embedding))]
    target._ds_compression_plan = []
    for tech in TECHNIQUES:
        tc = cc.get(tech, {})
        if not tc.get("shared_parameters", {}).get("enabled", False):
            continue
        for gname, shared, params, mods, related in _groups(tc):
            for n in names:
                if not _match(n, mods):
                    continue
                m = recursive_getattr(target, n)
                new = _to_compress(m)
                if new is None:
                    continue
                if new is not m:
                    recursive_setattr(target, n, new)
                target._ds_compression_plan.append((tech, n, shared, params, related))
    # techniques with schedule_offset 0 start immediately
    compression_scheduler(target, cc).step(0)
    return model


class compression_scheduler:
    """Enable each technique once the training step reaches its schedule_offset (reference `scheduler.py`)."""

    def __init__(self, model, compression_config):
        self.model = model
        self.cc = compression_config if "weight_quantization" in compression_config or not compression_config \
            else _cfg(compression_config)
        self.enabled = set()

    def step(self, step_zero_check=None):
        step = step_zero_check if step_zero_check is not None else getattr(self, "_step", 0)
        for (tech, n, shared, params, related) in getattr(self.model, "_ds_compression_plan", []):
            key = (tech, n)
            if key in self.enabled or step < shared.get("schedule_offset", 0):
                continue
            m = recursive_getattr(self.model, n)
            _enable(m, tech, shared, params)
            if hasattr(m, "update_masks"):
                m.update_masks()
            self.enabled.add(key)
        self._step = step + 1


@torch.no_grad()
def redundancy_clean(model, deepspeed_config, mpu=None):
    """Apply masks / quantisation permanently; row pruning shrinks the layer and its related consumers."""
    cc = _cfg(deepspeed_config)
    target = model.module if hasattr(model, "module") and isinstance(model.module, nn.Module) else model
    for (tech, n, shared, params, related) in getattr(target, "_ds_compression_plan", []):
        m = recursive_getattr(target, n)
        if tech == "weight_quantization" and hasattr(m, "fix_weight_quantization"):
            m.fix_weight_quantization()
        elif tech == "sparse_pruning" and getattr(m, "sparse_pruning_enabled", False):
            m.update_masks()
            m.fix_sparse_pruning_helper()
        elif tech == "row_pruning" and getattr(m, "row_pruning_enabled", False):
            m.update_masks()
            keep = m.fix_row_col_pruning_helper(dim_reduction=True)
            for rel_list in (related or []):
                for rn in rel_list:
                    for cand, cm in target.named_modules():
                        if isinstance(cm, nn.Linear) and _match(cand, [rn]) and cm.in_features == keep.numel():
                            if isinstance(cm, LinearLayer_Compress):
                                cm.fix_column_pruning(keep)
                            else:
                                cm.weight = nn.Parameter(cm.weight[:, keep].clone())
                                cm.in_features = int(keep.sum())
        elif tech == "head_pruning" and getattr(m, "head_pruning_enabled", False):
            m.update_masks()
            m.fix_head_pruning_helper(dim_reduction=False)
    return model


def student_initialization(student_model, teacher_model, deepspeed_config):
    """Copy the selected teacher layers (and other modules) into the student (reference `compress.py:186`)."""
    lr = _cfg(deepspeed_config).get("layer_reduction", {})
    prefix = lr["module_name_prefix"]
    t_layers = recursive_getattr(teacher_model, prefix)
    s_layers = recursive_getattr(student_model, prefix)
    for s_i, t_i in enumerate(lr["teacher_layer"]):
        s_layers[s_i].load_state_dict(t_layers[t_i].state_dict())
    for other in lr.get("other_module_name", []):
        recursive_getattr(student_model, other).load_state_dict(recursive_getattr(teacher_model, other).state_dict())
