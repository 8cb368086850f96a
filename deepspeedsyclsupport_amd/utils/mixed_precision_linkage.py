"""Low-precision <-> fp32-master linkage for flat partitions (reference `utils/mixed_precision_linkage.py:11-56`
`link_hp_params`, `utils/tensor_fragment.py:19-100,258-290` `tensor_fragment` / `get_hp_fragment_mapping`).

Contract: a list of low-precision (lp) parameters is thought of as one flat vector (parameters back to back in list
order); this rank owns the slice `[partition_start, partition_start + partition_size)` of the matching fp32 (hp) vector
as `flat_hp_partition`, with optimizer state tensors of the same shape. `link_hp_params` gives every lp parameter that
meets the slice an `_hp_mapping` describing the overlap — views into the lp parameter, the hp partition and each
optimizer state — and gives every lp parameter `get_full_hp_param` / `set_full_hp_param` / `get_full_hp_grad`
methods that assemble the whole tensor over `dp_group` (every rank contributes the elements it owns, summed by one
all-reduce).

The engine's own flat-group optimizer keeps this mapping in its group layout and serves `utils/tensor_fragment.py`'s
`safe_get_*` accessors from it; this module is the same facility for client code that manages its own flat partitions
(and for tools written against the reference's `_hp_mapping` attributes).
"""
import types
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from .. import comm as dist
from .tensor_fragment import (safe_get_full_fp32_param, safe_get_full_grad,  # noqa: F401
                              safe_get_full_optimizer_state, safe_get_local_fp32_param, safe_get_local_grad,
                              safe_get_local_optimizer_state, safe_set_full_fp32_param, safe_set_full_optimizer_state)


@dataclass
class fragment_address:
    numel: int
    start: int


@dataclass
class tensor_fragment:
    """The overlap of one lp parameter with this rank's hp partition."""
    lp_fragment: torch.Tensor
    lp_fragment_address: fragment_address
    hp_fragment: torch.Tensor
    hp_fragment_address: fragment_address
    optim_fragment: Dict[str, torch.Tensor]
    gradient_dict: Optional[dict]
    offload_gradient_dict: Optional[dict]
    use_offload: bool
    param_group_index: int

    def update_hp(self):
        self.hp_fragment.data.copy_(self.lp_fragment.data)

    def update_lp(self):
        self.lp_fragment.data.copy_(self.hp_fragment.data)

    def get_optim_state_keys(self):
        return list(self.optim_fragment.keys())

    def get_optim_state_fragment(self, key):
        if key not in self.optim_fragment:
            raise ValueError(f"{key} not found in optimizer state fragment")
        return self.optim_fragment[key]

    def get_hp_fragment_address(self):
        return self.hp_fragment_address

    def get_hp_fragment(self, optim_state_key=None):
        return self.hp_fragment if optim_state_key is None else self.get_optim_state_fragment(optim_state_key)


def _assemble(param, piece_of):
    """Full fp32 tensor of `param`: this rank's elements placed by `piece_of(mapping)`, the rest from its peers."""
    full = torch.zeros(param.numel(), dtype=torch.float32, device=param.device)
    m = getattr(param, "_hp_mapping", None)
    if m is not None:
        a = m.lp_fragment_address
        full.narrow(0, a.start, a.numel).copy_(piece_of(m).reshape(-1)[:a.numel] if piece_of(m).numel() == a.numel
                                               else piece_of(m).reshape(-1).narrow(0, a.start, a.numel))
    if dist.is_initialized():
        dist.all_reduce(full, group=param._dp_group)
    return full.view(param.shape)


def get_full_hp_param(self, optim_state_key=None):
    return _assemble(self, lambda m: m.get_hp_fragment(optim_state_key))


def set_full_hp_param(self, value, optim_state_key=None):
    m = getattr(self, "_hp_mapping", None)
    if m is not None:
        a = m.lp_fragment_address
        m.get_hp_fragment(optim_state_key).data.copy_(value.reshape(-1).narrow(0, a.start, a.numel))


def get_full_hp_grad(self):
    def grad_piece(m):
        grads = m.offload_gradient_dict if m.use_offload else m.gradient_dict
        if grads is None or grads.get(m.param_group_index) is None:
            raise ValueError("Gradients are only available immediately after backward and before engine step")
        # per group, the gradients of the parameters that meet this rank's partition, in list order: either the
        # whole parameter's gradient or just the owned fragment
        return grads[m.param_group_index][self._index_in_param_group].to(torch.float32)

    return _assemble(self, grad_piece)


def get_hp_fragment_mapping(lp_param, lp_start, flat_hp_partition, gradient_dict, offload_gradient_dict, use_offload,
                            param_group_index, partition_start, partition_size, optimizer_state_dict):
    lo = max(lp_start, partition_start)
    hi = min(lp_start + lp_param.numel(), partition_start + partition_size)
    if lo >= hi:
        raise AssertionError(f"parameter at [{lp_start}, {lp_start + lp_param.numel()}) does not meet the partition "
                             f"[{partition_start}, {partition_start + partition_size})")
    n = hi - lo
    hp_addr = fragment_address(numel=n, start=lo - partition_start)
    lp_addr = fragment_address(numel=n, start=lo - lp_start)
    optim = {k: v.narrow(0, hp_addr.start, n) for k, v in (optimizer_state_dict or {}).items()
             if torch.is_tensor(v) and v.shape == flat_hp_partition.shape}
    return tensor_fragment(lp_fragment=lp_param.detach().view(-1).narrow(0, lp_addr.start, n),
                           lp_fragment_address=lp_addr, hp_fragment=flat_hp_partition.narrow(0, hp_addr.start, n),
                           hp_fragment_address=hp_addr, optim_fragment=optim, gradient_dict=gradient_dict,
                           offload_gradient_dict=offload_gradient_dict, use_offload=use_offload,
                           param_group_index=param_group_index)


def link_hp_params(lp_param_list, flat_hp_partition, gradient_dict=None, offload_gradient_dict=None,
                   use_offload=False, param_group_index=0, partition_start=0, partition_size=None,
                   partition_optimizer_state=None, dp_group=None):
    """Attach `_hp_mapping` (or None when the parameter lies outside this rank's slice), `_dp_group`,
    `_index_in_param_group` and the full-tensor accessors to every parameter of `lp_param_list`. Returns the linked
    (parameter, flat offset) pairs."""
    if partition_size is None:
        partition_size = flat_hp_partition.numel()
    end = partition_start + partition_size
    linked, off, idx = [], 0, 0
    for p in lp_param_list:
        p._hp_mapping = None
        p._dp_group = dp_group
        p.get_full_hp_param = types.MethodType(get_full_hp_param, p)
        p.get_full_hp_grad = types.MethodType(get_full_hp_grad, p)
        p.set_full_hp_param = types.MethodType(set_full_hp_param, p)
        if off < end and off + p.numel() > partition_start:
            p._index_in_param_group = idx
            idx += 1
            p._hp_mapping = get_hp_fragment_mapping(p, off, flat_hp_partition, gradient_dict, offload_gradient_dict,
                                                    use_offload, param_group_index, partition_start, partition_size,
                                                    partition_optimizer_state)
            linked.append((p, off))
        off += p.numel()
    return linked
