"""Shard sizes for tensor-parallel slicing, with uneven splits when the key/value head count does not divide the
degree (reference `module_inject/tp_shard.py`): once `set_num_kv_heads` has been called, sizes are handed out in whole
kv-head units and the first `num_kv_heads % mp_size` ranks own one unit more."""
from .. import comm as dist

_state = {"num_kv_heads": None, "n_embd": None}


def set_num_kv_heads(num):
    _state["num_kv_heads"] = num


def get_num_kv_heads():
    return _state["num_kv_heads"]


def set_n_embd(num):
    _state["n_embd"] = num


def get_n_embd():
    return _state["n_embd"]


def get_shard_size(total_size, mp_size, rank=None):
    heads = _state["num_kv_heads"]
    if heads is None:
        if total_size % mp_size:
            raise AssertionError(f"Number of attention heads ({total_size}) must be divisible by mp_size ({mp_size})")
        return total_size // mp_size
    if rank is None:
        rank = dist.get_rank()
    units = heads // mp_size + (1 if rank < heads % mp_size else 0)
    return total_size * units // heads


def get_shard_size_list(total_size, mp_size):
    return [get_shard_size(total_size, mp_size, r) for r in range(mp_size)]
