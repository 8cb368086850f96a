"""Communication-compressed optimizers (reference `runtime/fp16/onebit/`)."""
from .adam import OnebitAdam
from .lamb import OnebitLamb
from .zoadam import ZeroOneAdam


def build_onebit_optimizer(name, model_parameters, engine, params):
    cls = {"onebitadam": OnebitAdam, "zerooneadam": ZeroOneAdam, "onebitlamb": OnebitLamb}[name.lower()]
    assert engine.zero_optimization_stage() == 0, f"{cls.__name__} needs ZeRO stage 0 (it owns the communication)"
    return cls(model_parameters, deepspeed=engine, **params)
