"""`_init_group_wise_weight_quantization` (reference `inference/quantization/quantization.py:20-111`): walk a built
model and swap every `nn.Linear` / `nn.Embedding` whose qualified name contains a configured key for its quantised
counterpart.

    ds_config = {"weight_quantization": {"post_init_quant": {
        "fc":                {"num_bits": 4, "group_size": 64, "group_dim": 1, "symmetric": False},
        "self_attn.q_proj":  {...}, ...}}}

`weight_quantization.quantized_initialization` (one config for every linear and embedding, reference
`runtime/zero/partition_parameters.py:317`) is the same pass with a key that matches every name; `deepspeed.initialize`
applies it before it builds the engine. Under ZeRO-3 a partitioned weight is gathered for the moment it is quantised;
the packed codes (4-8x smaller) then live whole on every rank as buffers.
"""
import gc
from collections import deque
from typing import Dict

from torch import nn

from ...utils.logging import logger
from . import layers
from .layers import QUANTIZATION_LAYER_MAPPINGS
from .utils import recursive_setattr


def _numel(module):
    w = module.weight
    return getattr(w, "ds_numel", w.numel())


def _init_group_wise_weight_quantization(model: nn.Module, ds_config: Dict) -> nn.Module:
    assert "weight_quantization" in ds_config, "Please provide quantization config in ds_config"
    wq = ds_config["weight_quantization"]
    quantization_config = dict(wq.get("post_init_quant") or {})
    if wq.get("quantized_initialization"):
        quantization_config[""] = wq["quantized_initialization"]  # "" is contained in every module name
    matched_by_key, count = {}, 0
    # small weights first, so the peak of (original + packed copy) is met with the least memory still unconverted
    todo = deque(sorted(((n, m) for n, m in model.named_modules() if type(m) in QUANTIZATION_LAYER_MAPPINGS),
                        key=lambda nm: _numel(nm[1])))
    while todo:
        name, module = todo.popleft()
        keys = [k for k in quantization_config if k in name and k != ""]
        assert len(keys) <= 1, f"{name} matched multiple quantization key word {keys}"
        key = keys[0] if keys else ("" if "" in quantization_config else None)
        if key is None:
            continue
        recursive_setattr(model, name, QUANTIZATION_LAYER_MAPPINGS[type(module)](quantization_config[key], module))
        matched_by_key.setdefault(key, []).append(name)
        count += 1
        del module
        gc.collect()
    layers.quantized_weight_registry.clear()
    logger.info(f"Group-wise weight quantization summary: convert {count} node(s) to quantized implementation")
    for key, names in matched_by_key.items():
        logger.info(f"Key: {key!r}, matched modules: " + ", ".join(names))
    return model
