"""Key names of the `compression_training` config section (reference `compression/constants.py`), built from the
defaults tables of `compression/config.py` so that the two cannot drift: for technique T with constant prefix P,
`P = "T"`, `P_<KEY> = "key"` and `P_<KEY>_DEFAULT = default`; choice values become `P_<KEY>_<VALUE>`."""
from .config import CHOICES, LAYER_REDUCTION_DEFAULTS, PARAM_DEFAULTS, SHARED_DEFAULTS

COMPRESSION_TRAINING = "compression_training"
SHARED_PARAMETERS = "shared_parameters"
DIFFERENT_GROUPS = "different_groups"
TECHNIQUE_ENABLED = "enabled"
TECHNIQUE_SCHEDULE_OFFSET = "schedule_offset"
TECHNIQUE_SCHEDULE_OFFSET_END = "schedule_offset_end"
DIFFERENT_GROUPS_PARAMETERS = "params"
DIFFERENT_GROUPS_MODULE_SCOPE = "modules"
DIFFERENT_GROUPS_MODULE_SCOPE_DEFAULT = "*"
DIFFERENT_GROUPS_RELATED_MODULE_SCOPE = "related_modules"
DIFFERENT_GROUPS_RELATED_MODULE_SCOPE_DEFAULT = None

LAYER_REDUCTION = "layer_reduction"
LAYER_REDUCTION_ENABLED = "enabled"
LAYER_REDUCTION_ENABLED_DEFAULT = LAYER_REDUCTION_DEFAULTS["enabled"]
for _k in LAYER_REDUCTION_DEFAULTS:
    if _k != "enabled":
        globals()[_k.upper()] = _k

# technique -> (name of the section constant, prefix of its key constants)
_PREFIX = {
    "weight_quantization": ("WEIGHT_QUANTIZATION", "WEIGHT_QUANTIZE"),
    "activation_quantization": ("ACTIVATION_QUANTIZATION", "ACTIVATION_QUANTIZE"),
    "sparse_pruning": ("SPARSE_PRUNING", "SPARSE_PRUNING"),
    "row_pruning": ("ROW_PRUNING", "ROW_PRUNING"),
    "head_pruning": ("HEAD_PRUNING", "HEAD_PRUNING"),
    "channel_pruning": ("CHANNEL_PRUNING", "CHANNEL_PRUNING"),
}
# config key -> the part of the constant's name after the prefix, where it is not just the key in capitals
_SUFFIX = {
    "quantizer_kernel": "KERNEL", "quantize_groups": "GROUPS", "quantize_verbose": "VERBOSE",
    "quantization_type": "TYPE", "quantize_weight_in_forward": "IN_FORWARD_ENABLED",
    "quantize_change_ratio": "CHANGE_RATIO", "range_calibration": "RANGE",
}
_VALUE_SUFFIX = {"stochastic": "STOCHASTIC_ROUNDING", "nearest": "NEAREST_ROUNDING"}


def _fill():
    g = globals()
    for tech, (section, pre) in _PREFIX.items():
        g[section] = tech
        for key, default in SHARED_DEFAULTS[tech].items():
            name = f"{pre}_{_SUFFIX.get(key, key.upper())}"
            g[name] = key
            g[f"{name}_DEFAULT"] = default
            for value in CHOICES.get((tech, key), ()):
                tail = _VALUE_SUFFIX.get(value, value.upper())
                g[f"{pre}_{tail}" if key in ("quantization_type", "rounding") else f"{name}_{tail}"] = value
        for key in PARAM_DEFAULTS[tech]:
            g[f"{pre}_{key.upper()}"] = key
    # names the pattern does not give
    g["ACTIVATION_QUANTIZATION_ENABLED"], g["ACTIVATION_QUANTIZATION_ENABLED_DEFAULT"] = "enabled", False
    g["WEIGHT_QUANTIZATION_PERIOD"] = "quantization_period"
    g["WEIGHT_QUANTIZATION_PERIOD_DEFAULT"] = PARAM_DEFAULTS["weight_quantization"]["quantization_period"]
    g["WEIGHT_QUANTIZE_FP16_MIXED_QUANTIZE_ENABLED"] = "enabled"
    g["WEIGHT_QUANTIZE_FP16_MIXED_QUANTIZE_ENABLED_DEFAULT"] = False
    g["HEAD_PRUNING_METHOD_L1"] = "l1"
    g["SPARSE_PRUNING_DENSE_RATIO_DEFAULT"] = 0.1
    g["SPARSE_PRUNING_SCHEDULE_OFFSET_END_DEFAULT"] = g["SPARSE_PRUNING_SCHEDULE_OFFSET_DEFAULT"]


_fill()
del _fill, _k
