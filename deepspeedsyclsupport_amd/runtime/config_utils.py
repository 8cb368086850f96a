"""Pydantic base for config sub-sections with deprecated-alias support (reference `runtime/config_utils.py:16-80`)."""
import collections
import json

from pydantic import BaseModel, ConfigDict


class DeepSpeedConfigModel(BaseModel):
    """Sub-config base: forbids unknown keys (typo protection), accepts field aliases such as `stage3_*`.

    """
    model_config = ConfigDict(extra="forbid", populate_by_name=True, validate_assignment=True,
                              arbitrary_types_allowed=True, protected_namespaces=())

    def __init__(self, strict=False, **data):
        # HF-style "auto" values mean "use the default" (reference config_utils.py:40)
        if not strict:
            data = {k: v for k, v in data.items() if (v != "auto" or k == "replace_method")}
        super().__init__(**data)


def get_scalar_param(param_dict, param_name, param_default_value):
    return param_dict.get(param_name, param_default_value)


def get_list_param(param_dict, param_name, param_default_value):
    return param_dict.get(param_name, param_default_value)


def get_dict_param(param_dict, param_name, param_default_value):
    return param_dict.get(param_name, param_default_value)


def dict_raise_error_on_duplicate_keys(ordered_pairs):
    d = dict((k, v) for k, v in ordered_pairs)
    if len(d) != len(ordered_pairs):
        counter = collections.Counter([pair[0] for pair in ordered_pairs])
        keys = [key for key, value in counter.items() if value > 1]
        raise ValueError(f"Duplicate keys in DeepSpeed config: {keys}")
    return d


class ScientificNotationEncoder(json.JSONEncoder):
    """Pretty-prints a config with numbers above 1000 in scientific notation (bucket sizes read as 5.000000e+08)
    — the reference's `print_configuration` output style. Implemented as a recursive formatter over the decoded
    structure; strings and other leaves go through the stock encoder."""

    def _leaf(self, o):
        if isinstance(o, bool):
            return "true" if o else "false"
        if isinstance(o, (int, float)):
            return f"{o:e}" if o > 1e3 else f"{o}"
        return json.JSONEncoder.encode(self, o)

    def _fmt(self, o, depth):
        step = self.indent if self.indent is not None else 4
        pad, inner = " " * (depth * step), " " * ((depth + 1) * step)
        if isinstance(o, collections.abc.Mapping):
            items = sorted(o.items()) if self.sort_keys else o.items()
            body = ", ".join(f'\n{inner}"{k}": {self._fmt(v, depth + 1)}' for k, v in items)
            return "{" + body + f"\n{pad}" + "}"
        if isinstance(o, collections.abc.Sequence) and not isinstance(o, (str, bytes)):
            return "[" + ", ".join(self._fmt(v, depth + 1) for v in o) + "]"
        return self._leaf(o)

    def encode(self, o):
        return self._fmt(o, 0)

    def iterencode(self, o, _one_shot=False):
        yield self.encode(o)


def get_config_default(config, field_name):
    """Default of a field of a config model class (it must have one)."""
    field = config.model_fields[field_name]
    assert not field.is_required(), f"'{field_name}' is a required field and does not have a default value"
    return field.get_default(call_default_factory=True)


class pp_int(int):
    """An int that prints with thousands separators (or as a custom string) in config dumps."""

    def __new__(cls, val, custom_print_str=None):
        inst = super().__new__(cls, val)
        inst.custom_print_str = custom_print_str
        return inst

    def __repr__(self):
        return self.custom_print_str if self.custom_print_str else f"{self.real:,}"


class DeepSpeedConfigObject:
    """Base of the plain (non-pydantic) config holders: printable as JSON."""

    def repr(self):
        return self.__dict__

    def __repr__(self):
        return json.dumps(self.__dict__, sort_keys=True, indent=4, cls=ScientificNotationEncoder)

