"""Low-precision <-> fp32-master linkage (reference `utils/mixed_precision_linkage.py:11` link_hp_params).

The flat ZeRO optimizer already records, for every 16-bit parameter, which slice of which fp32 master partition
holds it (`param.ds_group` / the group layout); `utils/tensor_fragment.py` reads full or local fp32 values, grads and
optimizer states through that mapping. These functions are the reference-named entry points onto it."""
from .tensor_fragment import (safe_get_full_fp32_param, safe_get_full_grad,  # noqa: F401
                              safe_get_full_optimizer_state, safe_get_local_fp32_param, safe_get_local_grad,
                              safe_get_local_optimizer_state, safe_set_full_fp32_param, safe_set_full_optimizer_state)


def link_hp_params(lp_param_list, flat_hp_partition=None, gradient_dict=None, offload_gradient_dict=None,
                   use_offload=False, param_group_index=0, partition_start=0, partition_size=0,
                   partition_optimizer_state=None, dp_group=None):
    """Return, per low-precision param, the (group, offset, numel) address of its fp32 master slice."""
    out = []
    for p in lp_param_list:
        g = getattr(p, "ds_group", None)
        out.append(None if g is None else (g.idx, getattr(p, "ds_offset", None), p.ds_numel if hasattr(p, "ds_numel")
                                           else p.numel()))
    return out
