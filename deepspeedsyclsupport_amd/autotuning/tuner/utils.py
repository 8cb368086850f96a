"""Feature encoding of tuning-space points (reference `autotuning/tuner/utils.py`)."""
import math

import numpy as np


def flatten(d, parent_key="", sep="_"):
    out = {}
    for k, v in d.items():
        key = f"{parent_key}{sep}{k}" if parent_key else k
        if isinstance(v, dict):
            out.update(flatten(v, key, sep))
        else:
            out[key] = v
    return out


def _num(v):
    if isinstance(v, bool):
        return float(v)
    if isinstance(v, (int, float)):
        return math.log2(v) if v > 0 else float(v)  # sizes span decades: log scale
    return float(abs(hash(v)) % 997) / 997.0


def dict_to_feature(feature_dict, keys):
    flat = flatten(feature_dict)
    return np.array([_num(flat.get(k, 0.0)) for k in keys], dtype=np.float64)
