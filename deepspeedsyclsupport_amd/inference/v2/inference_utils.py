"""Small enums and helpers shared by the ragged-inference modules (reference `inference/v2/inference_utils.py`)."""
from enum import Enum, IntEnum

import torch


class NormTypeEnum(Enum):
    LayerNorm = "layer_norm"
    RMSNorm = "rms_norm"


class DtypeEnum(Enum):
    """A dtype that can be looked up by the torch dtype or by any of its usual spellings: `DtypeEnum("bf16")`,
    `DtypeEnum(torch.bfloat16)` and `DtypeEnum("torch.bfloat16")` are the same member; `.value` is the torch dtype."""
    fp16 = torch.float16
    fp32 = torch.float32
    bf16 = torch.bfloat16
    int8 = torch.int8

    @classmethod
    def _missing_(cls, value):
        if isinstance(value, str):
            key = value.replace("torch.", "").lower()
            spelled = {"half": "fp16", "float16": "fp16", "float": "fp32", "float32": "fp32", "bfloat16": "bf16",
                       "bfloat": "bf16"}.get(key, key)
            if spelled in cls.__members__:
                return cls[spelled]
        return None


ELEM_SIZES = {dt: torch.empty((), dtype=dt).element_size()
              for dt in (torch.float16, torch.bfloat16, torch.float32, torch.float64, torch.int8, torch.uint8,
                         torch.int16, torch.int32, torch.int64, torch.bool)}


class ActivationType(IntEnum):
    InvalidType = -1
    GELU = 0
    RELU = 1
    SILU = 2
    GEGLU = 3
    ReGLU = 4
    SiGLU = 5
    IDENTITY = 6


_GATED = {ActivationType.GEGLU: "gelu", ActivationType.ReGLU: "relu", ActivationType.SiGLU: "silu"}
_PLAIN = {ActivationType.GELU: "gelu", ActivationType.RELU: "relu", ActivationType.SILU: "silu",
          ActivationType.IDENTITY: "identity"}


def is_gated(act_fn: ActivationType) -> bool:
    return ActivationType(act_fn) in _GATED


def act_name(act_fn: ActivationType) -> str:
    """The activation name the in-tree kernels take ("gelu" / "relu" / "silu" / "identity")."""
    act_fn = ActivationType(act_fn)
    return _GATED.get(act_fn) or _PLAIN[act_fn]


def elem_size(dtype: torch.dtype) -> int:
    try:
        return ELEM_SIZES[dtype]
    except KeyError:
        raise ValueError(f"Unknown dtype size for {dtype}")


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)
