"""A tensor that carries named auxiliary tensors (scales of a quantised weight, ...) through `.to()` and friends
(reference `inference/v2/inference_parameter.py`). Model code treats it as the weight; kernels that know about an
auxiliary attribute read it by name."""
from typing import Dict

import torch

CORE_PARAM = "_ds_core_param_key"
STR_TO_DTYPE = {"torch.float32": torch.float32, "torch.float64": torch.float64, "torch.float16": torch.float16,
                "torch.bfloat16": torch.bfloat16, "torch.int64": torch.int64, "torch.int32": torch.int32,
                "torch.int16": torch.int16, "torch.int8": torch.int8, "torch.uint8": torch.uint8,
                "torch.bool": torch.bool}


class InferenceParameter(torch.Tensor):

    @staticmethod
    def __new__(cls, tensor, *args, **kwargs):
        new = super().__new__(cls, tensor, *args, **kwargs)
        if hasattr(tensor, "_aux_attrs"):
            setattr(new, "_aux_attrs", tensor.aux_attrs)
        return new

    def to(self, *args, **kwargs):
        new = InferenceParameter.initialize(super().to(*args, **kwargs))
        for name, attr in getattr(self, "_aux_attrs", {}).items():
            moved = attr.to(*args, **kwargs)
            setattr(new, name, moved)
            new._aux_attrs[name] = moved
        return new

    @classmethod
    def initialize(cls, core_param: torch.Tensor, **kwargs) -> "InferenceParameter":
        param = InferenceParameter(core_param)
        param._aux_attrs = dict(kwargs)
        for name, attr in kwargs.items():
            if hasattr(param, name):
                raise ValueError(f"Attribute {name} already exists on param.")
            if not isinstance(attr, torch.Tensor):
                raise ValueError(f"Attribute {name} must be a tensor.")
            setattr(param, name, attr)
        return param

    @classmethod
    def initialize_raw(cls, **kwargs) -> "InferenceParameter":
        if CORE_PARAM not in kwargs:
            raise ValueError(f"Must provide core parameter, with key {CORE_PARAM}.")
        aux = {k: v for k, v in kwargs.items() if k != CORE_PARAM}
        return cls.initialize(kwargs[CORE_PARAM], **aux)

    @property
    def aux_attrs(self) -> Dict[str, torch.Tensor]:
        return self._aux_attrs
