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

from .basic_layer import BNLayer_Compress, Conv2dLayer_Compress, LinearLayer_Compress
from .config import TECHNIQUES, get_compression_config
from .helper import fix_compression, recursive_getattr, recursive_setattr, to_compress_module  # noqa: F401
from .scheduler import compression_scheduler  # noqa: F401

# which module types each technique applies to
_APPLIES = {
    "weight_quantization": (nn.Linear, nn.Embedding, nn.Conv2d),
    "activation_quantization": (nn.Linear, nn.Conv2d),
    "sparse_pruning": (nn.Linear, ),
    "row_pruning": (nn.Linear, ),
    "head_pruning": (nn.Linear, ),
    "channel_pruning": (nn.Conv2d, ),
}


def _cfg(deepspeed_config):
    if isinstance(deepspeed_config, str):
        with open(deepspeed_config) as f:
            deepspeed_config = json.load(f)
    if hasattr(deepspeed_config, "_param_dict"):
        deepspeed_config = deepspeed_config._param_dict
    return get_compression_config(deepspeed_config)


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


def _layer_reduction(model, lr, teacher_model=None):
    if not lr.get("enabled", False):
        return
    prefix = lr["module_name_prefix"]
    keep = lr.get("teacher_layer") or list(range(lr["keep_number_layer"]))
    layers = recursive_getattr(model, prefix)
    recursive_setattr(model, prefix, nn.ModuleList([layers[i] for i in keep]))


def init_compression(model, deepspeed_config, teacher_model=None, mpu=None):
    """Swap the modules named by each enabled technique's groups for their compression-aware versions and record
    the plan the scheduler enables (techniques at schedule_offset 0 start immediately). With a teacher model and
    layer reduction, the student is initialised from the selected teacher layers."""
    cc = _cfg(deepspeed_config)
    target = model.module if hasattr(model, "module") and isinstance(model.module, nn.Module) else model
    lr = cc["layer_reduction"]
    if lr["enabled"] and teacher_model is not None:
        student_initialization(target, teacher_model, deepspeed_config)
    else:
        _layer_reduction(target, lr)
    target._ds_compression_plan = []
    for tech in TECHNIQUES:
        tc = cc[tech]
        shared = tc["shared_parameters"]
        if not shared.get("enabled", False):
            continue
        excluded = shared.get("excluded_modules") or []
        for gname, g in tc["different_groups"].items():
            for n, m in list(target.named_modules()):
                if not n or not isinstance(m, _APPLIES[tech]) or not _match(n, g["modules"]) or _match(n, excluded):
                    continue
                new = to_compress_module(m, mpu)
                if new is None:
                    continue
                if new is not m:
                    recursive_setattr(target, n, new)
                target._ds_compression_plan.append((tech, n, shared, g["params"], g["related_modules"]))
    compression_scheduler(target, cc).step(0)
    return model


def _related(target, patterns, kinds):
    for rn in patterns:
        for cand, cm in target.named_modules():
            if cand and isinstance(cm, kinds) and _match(cand, [rn]):
                yield cand, cm


@torch.no_grad()
def redundancy_clean(model, deepspeed_config, mpu=None):
    """Apply masks / quantisation permanently. Row pruning shrinks the layer and the consumers named in
    `related_modules` (their input columns); channel pruning shrinks the conv, its BatchNorm and the next conv's
    input channels (`related_modules`)."""
    target = model.module if hasattr(model, "module") and isinstance(model.module, nn.Module) else model
    for (tech, n, shared, params, related) in getattr(target, "_ds_compression_plan", []):
        m = recursive_getattr(target, n)
        if tech in ("weight_quantization", "sparse_pruning"):
            fix_compression(target, n, tech)
        elif tech == "row_pruning" and getattr(m, "row_pruning_enabled", False):
            keep = fix_compression(target, n, tech, dim_reduction=True)
            for rel_list in (related or []):
                for cand, cm in _related(target, rel_list, (nn.Linear, )):
                    if cm.in_features != keep.numel():
                        continue
                    if isinstance(cm, LinearLayer_Compress):
                        cm.fix_column_pruning(keep)
                    else:
                        cm.weight = nn.Parameter(cm.weight[:, keep].clone())
                        cm.in_features = int(keep.sum())
        elif tech == "head_pruning" and getattr(m, "head_pruning_enabled", False):
            fix_compression(target, n, tech, dim_reduction=False)
        elif tech == "channel_pruning" and getattr(m, "channel_pruning_enabled", False):
            keep = fix_compression(target, n, tech, dim_reduction=True)
            for rel_list in (related or []):
                for cand, cm in _related(target, rel_list, (nn.Conv2d, nn.BatchNorm2d)):
                    if isinstance(cm, nn.BatchNorm2d) and cm.num_features == keep.numel():
                        bn = cm if isinstance(cm, BNLayer_Compress) else to_compress_module(cm)
                        if bn is not cm:
                            recursive_setattr(target, cand, bn)
                        bn.fix_channel_pruning_helper(keep, dim_reduction=True)
                    elif isinstance(cm, nn.Conv2d) and cm.in_channels == keep.numel():
                        cv = cm if isinstance(cm, Conv2dLayer_Compress) else to_compress_module(cm)
                        if cv is not cm:
                            recursive_setattr(target, cand, cv)
                        cv.fix_channel_pruning_helper(mask=keep, dim_reduction=True)
    return model


def student_initialization(student_model, teacher_model, deepspeed_config):
    """Copy the selected teacher layers (and other modules) into the student (reference `compress.py:192`)."""
    lr = _cfg(deepspeed_config)["layer_reduction"]
    prefix = lr["module_name_prefix"]
    t_layers = recursive_getattr(teacher_model, prefix)
    s_layers = recursive_getattr(student_model, prefix)
    teacher_layer = lr["teacher_layer"] or list(range(lr["keep_number_layer"]))
    if len(s_layers) != len(teacher_layer):  # student still has the teacher's depth: reduce it first
        recursive_setattr(student_model, prefix, nn.ModuleList([s_layers[i] for i in teacher_layer]))
        s_layers = recursive_getattr(student_model, prefix)
    for s_i, t_i in enumerate(teacher_layer):
        s_layers[s_i].load_state_dict(t_layers[t_i].state_dict())
    for other in lr.get("other_module_name", []) or []:
        recursive_getattr(student_model, other).load_state_dict(recursive_getattr(teacher_model, other).state_dict())
