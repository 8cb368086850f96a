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

    def iterencode(self, o, _one_shot=False, level=0):
        indent = self.indent if self.indent is not None else 4
        prefix_close = " " * level * indent
        level += 1
        prefix = " " * level * indent
        if isinstance(o, bool):
            return "true" if o else "false"
        elif isinstance(o, float) or isinstance(o, int):
            if o > 1e3:
                return f"{o:e}"
            return f"{o}"
        elif isinstance(o, collections.abc.Mapping):
            x = [f'\n{prefix}"{k}": {self.iterencode(v, level=level)}' for k, v in o.items()]
            return "{" + ", ".join(x) + f"\n{prefix_close}" + "}"
        elif isinstance(o, collections.abc.Sequence) and not isinstance(o, str):
            return f"[{', '.join(map(self.iterencode, o))}]"
        return "\n, ".join(super().iterencode(o, _one_shot))
