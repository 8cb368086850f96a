"""Declarative checkpoint parameters (reference `inference/v2/model_implementations/parameter_base.py`).

A `ParameterBase` subclass declares the checkpoint tensors it is made of as class annotations — `params:
torch.Tensor`, or `experts: ParamList("n_experts")` for one tensor per expert — and `finalize()` turns them into the
entries of the canonical layer dict the injected model is loaded from (`inference/model_implementations/convert.py`:
q_w / k_w / v_w / o_w / gate_w / up_w / fc1_w / fc2_w / ln1_w ...). The owning container calls `finalize()` once
every declared tensor has arrived; a parameter whose tensors never arrive (an absent bias) contributes nothing.
"""
from typing import Dict

import torch


class ParamList:
    """Annotation marker: a list of tensors whose length is `getattr(model, count_attr)`."""

    def __init__(self, count_attr: str):
        self.count_attr = count_attr


ParametrizedList = ParamList


class ParameterBase:
    key = None  # canonical key for single-tensor parameters (set by `single(...)` subclasses)

    def __init__(self, model=None, name=None):
        self.inference_model = model
        self.name = name
        self._fields = {}
        for cls in reversed(type(self).__mro__):
            for field, ann in getattr(cls, "__annotations__", {}).items():
                if ann is torch.Tensor:
                    self._fields[field] = None
                elif isinstance(ann, ParamList):
                    n = getattr(model, ann.count_attr)
                    self._fields[field] = [None] * int(n)
        if not self._fields:
            raise TypeError(f"{type(self).__name__} declares no tensor fields")

    # ------------------------------------------------------------------------------------------ filling
    def set_field(self, field: str, tensor: torch.Tensor, index=None):
        if field not in self._fields:
            raise KeyError(f"{type(self).__name__} has no field {field!r}")
        slot = self._fields[field]
        if isinstance(slot, list):
            if index is None:
                raise ValueError(f"{type(self).__name__}.{field} is a list: the mapping needs a '*' index")
            slot[index] = tensor
        else:
            self._fields[field] = tensor

    def __getattr__(self, item):
        fields = self.__dict__.get("_fields", {})
        if item in fields:
            return fields[item]
        raise AttributeError(item)

    @property
    def touched(self) -> bool:
        return any((any(t is not None for t in v) if isinstance(v, list) else v is not None)
                   for v in self._fields.values())

    @property
    def complete(self) -> bool:
        return all((all(t is not None for t in v) if isinstance(v, list) else v is not None)
                   for v in self._fields.values())

    def finalize(self) -> Dict[str, torch.Tensor]:
        if self.key is None:
            raise NotImplementedError()
        return {self.key: self.params}


def single(key: str, doc: str = ""):
    """A parameter class made of one tensor `params` that lands under canonical key `key`."""

    class _Single(ParameterBase):
        params: torch.Tensor

    _Single.key = key
    _Single.__doc__ = doc or f"One tensor stored as `{key}`."
    return _Single
