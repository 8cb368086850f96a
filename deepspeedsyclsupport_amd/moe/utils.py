"""MoE helpers (reference `moe/utils.py`): detect expert params and split optimizer param groups so expert params
reduce over the expert-data-parallel group."""
from typing import Dict, List

import torch


def is_moe_param(param) -> bool:
    return hasattr(param, "allreduce") and not param.allreduce


def has_moe_layers(m):
    from .layer import MoE
    for mod in m.modules():
        if isinstance(mod, MoE):
            return True, mod.num_experts
    return False, 0


def split_params_into_shared_and_expert_params(params):
    shared, expert = [], []
    for p in params:
        (expert if is_moe_param(p) else shared).append(p)
    return shared, expert


def split_params_grads_into_shared_and_expert_params(group):
    shared, expert = [], []
    for p in group:
        if p.grad is not None:
            (expert if is_moe_param(p) else shared).append(p.grad.to(p.dtype))
    return shared, expert


def split_params_into_different_moe_groups_for_optimizer(param_groups, max_group_size=178956971):
    """Each input group becomes [dense group] + one group per expert-parallel group name ({'moe': True, 'name': ..})."""
    if isinstance(param_groups, dict):
        param_groups = [param_groups]
    elif not isinstance(param_groups, (list, tuple)):
        param_groups = [{"params": list(param_groups)}]
    out = []
    for g in param_groups:
        if g.get("moe", False):
            out.append(g)
            continue
        params = list(g["params"])
        dense = [p for p in params if not is_moe_param(p)]
        by_name: Dict[str, List] = {}
        for p in params:
            if is_moe_param(p):
                by_name.setdefault(p.group_name, []).append(p)
        base = {k: v for k, v in g.items() if k != "params"}
        out.append({**base, "params": dense})
        for name, ps in by_name.items():
            out.append({**base, "params": ps, "moe": True, "name": name})
    return [g for g in out if len(g["params"]) > 0]


def configure_moe_param_groups(model_parameters):
    return split_params_into_different_moe_groups_for_optimizer(model_parameters)
