"""`compression_training` config parsing with the reference defaults (reference `compression/config.py`,
`compression/constants.py`): every technique gets its `shared_parameters` filled in and its `different_groups`
validated (each group needs `params` and `modules`), so the rest of the package reads plain dicts."""
import copy

TECHNIQUES = ("weight_quantization", "activation_quantization", "sparse_pruning", "row_pruning", "head_pruning",
              "channel_pruning")

SHARED_DEFAULTS = {
    "weight_quantization": {"enabled": False, "quantizer_kernel": False, "schedule_offset": 0, "quantize_groups": 1,
                            "quantize_verbose": False, "quantization_type": "symmetric",
                            "quantize_weight_in_forward": False, "rounding": "nearest", "fp16_mixed_quantize": False,
                            "quantize_change_ratio": 0.001},
    "activation_quantization": {"enabled": False, "quantization_type": "symmetric", "range_calibration": "dynamic",
                                "schedule_offset": 1000},
    "sparse_pruning": {"enabled": False, "method": "l1", "schedule_offset": 1000, "schedule_offset_end": None,
                       "schedule_offset_stride": 1, "block_pattern": "4x1", "excluded_modules": []},
    "row_pruning": {"enabled": False, "method": "l1", "schedule_offset": 1000},
    "head_pruning": {"enabled": False, "method": "topk", "schedule_offset": 1000, "num_heads": None},
    "channel_pruning": {"enabled": False, "method": "l1", "schedule_offset": 1000},
}
PARAM_DEFAULTS = {
    "weight_quantization": {"start_bits": 8, "target_bits": 8, "quantization_period": 1},
    "activation_quantization": {"bits": 8},
    "sparse_pruning": {"dense_ratio": 0.5},
    "row_pruning": {"dense_ratio": 0.5},
    "head_pruning": {"dense_ratio": 0.5},
    "channel_pruning": {"dense_ratio": 0.5},
}
LAYER_REDUCTION_DEFAULTS = {"enabled": False, "keep_number_layer": None, "module_name_prefix": "",
                            "teacher_layer": None, "other_module_name": []}
CHOICES = {
    ("weight_quantization", "quantization_type"): ("symmetric", "asymmetric"),
    ("weight_quantization", "rounding"): ("nearest", "stochastic"),
    ("activation_quantization", "quantization_type"): ("symmetric", "asymmetric"),
    ("activation_quantization", "range_calibration"): ("dynamic", "static"),
    ("sparse_pruning", "method"): ("l1", "topk", "snip_momentum"),
    ("row_pruning", "method"): ("l1", "topk"),
    ("head_pruning", "method"): ("topk", ),
    ("channel_pruning", "method"): ("l1", "topk"),
}


def get_compression_config(param_dict):
    """Normalised `compression_training` section of a DeepSpeed config dict (or the section itself)."""
    cc = param_dict.get("compression_training", param_dict) if isinstance(param_dict, dict) else {}
    out = {}
    for tech in TECHNIQUES:
        raw = cc.get(tech, {}) or {}
        shared = copy.deepcopy(SHARED_DEFAULTS[tech])
        shared.update(raw.get("shared_parameters", {}) or {})
        for (t, key), allowed in CHOICES.items():
            if t == tech and shared.get(key) not in allowed:
                raise ValueError(f"compression_training.{tech}.{key} must be one of {allowed}, got {shared.get(key)}")
        if tech == "head_pruning" and shared["enabled"] and not shared.get("num_heads"):
            raise ValueError("compression_training.head_pruning needs shared_parameters.num_heads")
        groups = {}
        for name, g in (raw.get("different_groups", {}) or {}).items():
            if "params" not in g or "modules" not in g:
                if shared["enabled"]:
                    raise ValueError(f"compression_training.{tech}.different_groups.{name} needs 'params' and "
                                     "'modules'")
            params = copy.deepcopy(PARAM_DEFAULTS[tech])
            params.update(g.get("params", {}) or {})
            if tech == "weight_quantization" and params["target_bits"] > params["start_bits"]:
                raise ValueError("weight_quantization target_bits must not exceed start_bits")
            if "dense_ratio" in params and not 0.0 < float(params["dense_ratio"]) <= 1.0:
                raise ValueError(f"{tech} dense_ratio must be in (0, 1]")
            groups[name] = {"params": params, "modules": list(g.get("modules", ["*"])),
                            "related_modules": g.get("related_modules")}
        out[tech] = {"shared_parameters": shared, "different_groups": groups}
    lr = copy.deepcopy(LAYER_REDUCTION_DEFAULTS)
    lr.update(cc.get("layer_reduction", {}) or {})
    if lr["enabled"] and not lr["module_name_prefix"]:
        raise ValueError("compression_training.layer_reduction needs module_name_prefix")
    if lr["enabled"] and lr["teacher_layer"] is None and lr["keep_number_layer"] is None:
        raise ValueError("compression_training.layer_reduction needs teacher_layer or keep_number_layer")
    out["layer_reduction"] = lr
    return out
