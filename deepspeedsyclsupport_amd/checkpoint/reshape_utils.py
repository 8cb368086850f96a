"""File discovery and state merging helpers for 3-D (pipeline x tensor x data parallel) checkpoint folders
(reference `checkpoint/reshape_utils.py:12-98`)."""
import os
import re

import torch

from . import constants as CK


def basic_folder_validation(dir):
    if not os.path.exists(dir):
        raise FileNotFoundError(f"{dir} path does not exist")
    if not os.path.isdir(dir):
        raise NotADirectoryError(f"{dir} is not a folder")


def _natural(path):
    """Sort key that orders embedded integers numerically (…rank_2… before …rank_10…)."""
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]


def get_files(dir):
    out = []
    for root, _, files in os.walk(dir):
        out.extend(os.path.join(root, f) for f in files)
    return sorted(out, key=lambda p: (os.path.dirname(p), _natural(p)))


def get_files_with_prefix(all_files, prefix):
    return [f for f in all_files if os.path.basename(f).startswith(prefix)]


def validate_files(file_list):
    missing = [f for f in file_list if not os.path.isfile(f)]
    if missing:
        raise FileNotFoundError(f"missing checkpoint files: {missing[:3]}")


def get_zero_files(dir):
    files = get_files(dir)
    for prefix in (CK.ZERO_FILE_PREFIX, CK.FP16_ZERO_FILE_PREFIX, CK.BF16_ZERO_FILE_PREFIX):
        hit = [f for f in get_files_with_prefix(files, prefix) if f.endswith(CK.OPTIM_FILE_SUFFIX)]
        if hit:
            return hit
    return []


def partition_data(data_list, num_partitions):
    n = len(data_list)
    if n % num_partitions:
        raise ValueError(f"{n} items do not split into {num_partitions} equal partitions")
    k = n // num_partitions
    return [list(data_list[i * k:(i + 1) * k]) for i in range(num_partitions)]


def merge_state(a, b, key_list=()):
    """Structural merge of two states: tensors concatenate on dim 0, lists / tuples merge element-wise, dicts
    key-wise, anything else must agree (the first value is kept)."""
    if type(a) is not type(b):
        raise TypeError(f"cannot merge {type(a)} with {type(b)} at {'.'.join(map(str, key_list))}")
    if isinstance(a, dict):
        return {k: merge_state(a[k], b[k], (*key_list, k)) if k in b else a[k] for k in a}
    if isinstance(a, (list, tuple)):
        if len(a) != len(b):
            raise ValueError(f"length mismatch at {'.'.join(map(str, key_list))}: {len(a)} vs {len(b)}")
        return type(a)(merge_state(x, y, (*key_list, i)) for i, (x, y) in enumerate(zip(a, b)))
    if torch.is_tensor(a):
        return torch.cat([a, b], 0)
    return a


merge_state_dict = merge_state
merge_state_list = merge_state
