"""Tuning-space helpers (reference `autotuning/utils.py`): a tuning space is a (nested) config dict whose list
values are the candidate settings; `get_all_configs` expands the cartesian product, `canonical_name` names an
experiment by its tuned values, `prune_configs` removes duplicates."""
import copy
import itertools
import json


def get_tuning_keys(tuning_space, prefix=""):
    """Dotted paths of every list-valued (tuned) entry."""
    keys = []
    for k, v in tuning_space.items():
        path = f"{prefix}{k}"
        if isinstance(v, dict):
            keys += get_tuning_keys(v, path + ".")
        elif isinstance(v, list) and len(v) > 1:
            keys.append(path)
    return keys


def gen_combinations(d):
    """Cartesian product over the list values of a nested dict (non-lists are fixed)."""
    keys, choices = [], []
    for k, v in d.items():
        keys.append(k)
        if isinstance(v, dict):
            choices.append(list(gen_combinations(v)))
        elif isinstance(v, list):
            choices.append(v)
        else:
            choices.append([v])
    for combo in itertools.product(*choices):
        yield dict(zip(keys, combo))


def get_all_configs(tuning_space, ignore_keys=None):
    configs = list(gen_combinations(tuning_space))
    return prune_configs(configs, ignore_keys or [])


def _flat(d, prefix=""):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update(_flat(v, f"{prefix}{k}."))
        else:
            out[f"{prefix}{k}"] = v
    return out


def prune_configs(configs, ignored_keys=()):
    seen, out = set(), []
    for c in configs:
        flat = {k: v for k, v in _flat(c).items() if k not in ignored_keys}
        key = json.dumps(flat, sort_keys=True, default=str)
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def get_val_by_key(d, dotted):
    for part in dotted.split("."):
        d = d[part]
    return d


def set_val_by_key(d, dotted, v):
    parts = dotted.split(".")
    for part in parts[:-1]:
        d = d.setdefault(part, {})
    d[parts[-1]] = v


def _short(v):
    if isinstance(v, bool):
        return "T" if v else "F"
    if isinstance(v, (int, float)) and abs(v) >= 1e4:
        return f"{v:.0e}".replace("+0", "").replace("+", "")
    return str(v)


def canonical_name(config, tuning_keys=None, prefix=""):
    """'z3_mbs8_reduce_bucket_size5e8_overlap_commT'-style experiment name."""
    parts = [prefix] if prefix else []
    zo = config.get("zero_optimization", {})
    if "stage" in zo:
        parts.append(f"z{zo['stage']}")
    if "train_micro_batch_size_per_gpu" in config:
        parts.append(f"mbs{config['train_micro_batch_size_per_gpu']}")
    for k in tuning_keys or []:
        if k in ("zero_optimization.stage", "train_micro_batch_size_per_gpu"):
            continue
        try:
            parts.append(f"{k.split('.')[-1]}{_short(get_val_by_key(config, k))}")
        except KeyError:
            pass
    return "_".join(parts)


def merge(base, override):
    out = copy.deepcopy(base)
    for k, v in override.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out
