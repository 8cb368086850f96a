"""Containers that map checkpoint names onto declarative parameters (reference
`inference/v2/model_implementations/layer_container_base.py`).

A container class annotates its parameters (`qkv_w: UnfusedQKVParameter`) and lists, in `PARAM_MAPPING`, which
checkpoint tensor feeds which field: `"self_attn.q_proj.weight": "qkv_w.q_params"`. A `*` in a name stands for an
index (`experts.*.w1.weight` fills entry i of a `ParamList` field); a leading `*` matches any prefix; a list of
targets feeds one tensor to several fields (tied embeddings). `set_dependency(name, tensor)` is called with the name
relative to the container's prefix.
"""
import re
from typing import Dict

import torch

from .parameter_base import ParameterBase

MAPPING_KEY = "PARAM_MAPPING"


class LayerContainer:
    PARAM_MAPPING: Dict = {}

    def __init__(self, model=None) -> None:
        self.inference_model = model
        self._params = {}
        for cls in reversed(type(self).__mro__):
            for attr, ann in getattr(cls, "__annotations__", {}).items():
                if isinstance(ann, type) and issubclass(ann, ParameterBase):
                    self._params[attr] = ann(model, attr)
        self._patterns = []
        for src, targets in type(self).PARAM_MAPPING.items():
            targets = [targets] if isinstance(targets, str) else list(targets)
            for t in targets:
                attr, _, field = t.partition(".")
                if attr not in self._params:
                    raise ValueError(f"{type(self).__name__}: mapping target {t!r} names no annotated parameter")
                if field not in self._params[attr]._fields:
                    raise ValueError(f"{type(self).__name__}: {attr} has no field {field!r}")
            rx = re.escape(src).replace(r"\*", r"(.*?)")
            self._patterns.append((re.compile("^" + rx + "$"), src.startswith("*"), targets))

    def __getattr__(self, item):
        params = self.__dict__.get("_params", {})
        if item in params:
            return params[item]
        raise AttributeError(item)

    def set_dependency(self, dep_name: str, dep_value: torch.Tensor) -> bool:
        """Hand a checkpoint tensor to the field(s) its name maps to. Returns False when no pattern matches."""
        for rx, prefixed, targets in self._patterns:
            m = rx.match(dep_name)
            if not m:
                continue
            groups = list(m.groups())
            if prefixed and groups:
                groups = groups[1:]
            index = int(groups[0]) if groups and groups[0].isdigit() else None
            for t in targets:
                attr, _, field = t.partition(".")
                self._params[attr].set_field(field, dep_value, index)
            return True
        return False

    @property
    def is_initialized(self) -> bool:
        """Every parameter that has received anything has received everything, and at least one has."""
        touched = [p for p in self._params.values() if p.touched]
        return bool(touched) and all(p.complete for p in touched)

    def missing(self):
        return [f"{a}.{f}" for a, p in self._params.items() if p.touched and not p.complete
                for f, v in p._fields.items() if v is None or (isinstance(v, list) and any(t is None for t in v))]

    def canonical(self) -> Dict[str, torch.Tensor]:
        """Merged `finalize()` of the complete parameters: a canonical layer (or top-level) dict."""
        out = {}
        for p in self._params.values():
            if p.complete:
                out.update(p.finalize())
        return out

    def release(self):
        for p in self._params.values():
            for f, v in p._fields.items():
                p._fields[f] = [None] * len(v) if isinstance(v, list) else None
