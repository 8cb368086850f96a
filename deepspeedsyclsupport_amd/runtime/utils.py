"""Runtime helpers (reference `runtime/utils.py:195-1041`): global gradient norms / clipping across model- and
data-parallel groups, overflow checks, balanced partitioning, tensor alignment, memory reporting."""
import gc
import math

import torch

from .. import comm as dist
from ..accelerator import get_accelerator
from ..utils.logging import logger


def noop_decorator(func):
    return func


def ensure_directory_exists(filename):
    import os
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)


def set_random_seed(seed):
    import random

    import numpy as np
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    get_accelerator().manual_seed_all(seed)


def is_model_parallel_parameter(p):
    return bool(getattr(p, "model_parallel", False) or getattr(p, "tensor_model_parallel", False))


def _is_moe(p):
    return hasattr(p, "allreduce") and not p.allreduce


@torch.no_grad()
def get_global_norm_of_tensors(input_tensors, norm_type=2, mpu=None, use_graph=False, moe_ep_group=None):
    """Global norm of tensors spread over model-parallel ranks (sum of squares reduced over the MP group)."""
    tensors = [t for t in input_tensors if t is not None]
    if not tensors:
        return 0.0
    dev = tensors[0].device
    if norm_type == math.inf:
        total = torch.stack([t.detach().abs().max().float() for t in tensors]).max()
        if mpu is not None:
            dist.all_reduce(total, op=dist.ReduceOp.MAX, group=mpu.get_model_parallel_group())
        return float(total)
    total = torch.zeros((), dtype=torch.float32, device=dev)
    for t in tensors:
        total += t.detach().float().norm(norm_type)**norm_type
    if mpu is not None:
        dist.all_reduce(total, group=mpu.get_model_parallel_group())
    if moe_ep_group is not None:
        dist.all_reduce(total, group=moe_ep_group)
    return float(total)**(1.0 / norm_type)


@torch.no_grad()
def clip_grad_norm_(parameters, max_norm, norm_type=2, mpu=None):
    """Clip gradients; model-parallel duplicates are counted once (reference `utils.py:342`)."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return 0.0
    grads = [p.grad for p in params if (mpu is None or is_model_parallel_parameter(p) or
                                        mpu.get_model_parallel_rank() == 0)]
    total = get_global_norm_of_tensors(grads, norm_type, mpu)
    coef = max_norm / (total + 1e-6)
    if coef < 1:
        for p in params:
            p.grad.mul_(coef)
    return total


def get_grad_norm(parameters, norm_type=2, mpu=None):
    params = [p for p in parameters if p.grad is not None]
    return get_global_norm_of_tensors([p.grad for p in params], norm_type, mpu)


def get_weight_norm(parameters, norm_type=2, mpu=None):
    return get_global_norm_of_tensors([p.data for p in parameters], norm_type, mpu)


class CheckOverflow:
    """inf / nan detection in gradients, reduced over the data- (and model-) parallel groups."""

    def __init__(self, param_groups=None, mpu=None, zero_reduce_scatter=False, deepspeed=None):
        self.mpu = mpu
        self.params = [p for g in (param_groups or []) for p in g] if param_groups else []
        self.deepspeed = deepspeed

    @staticmethod
    def _has_inf_or_nan(x):
        s = float(x.float().sum())
        return s in (float("inf"), -float("inf")) or s != s

    def has_overflow_serial(self, params):
        return any(p.grad is not None and self._has_inf_or_nan(p.grad.data) for p in params)

    def has_overflow(self, params, has_moe_params=None):
        overflow = self.has_overflow_serial(params)
        flag = torch.tensor([1.0 if overflow else 0.0], device=get_accelerator().current_device_name()
                            if get_accelerator().device_name() != "cpu" else "cpu")
        if dist.is_initialized():
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return bool(flag.item())

    def check(self, param_groups=None):
        params = [p for g in param_groups for p in g] if param_groups else self.params
        return self.has_overflow(params)


def partition_uniform(num_items, num_parts):
    parts = [0] * (num_parts + 1)
    if num_items <= num_parts:
        for p in range(num_parts + 1):
            parts[p] = min(p, num_items)
        return parts
    chunk = num_items // num_parts
    rem = num_items % num_parts
    for p in range(1, num_parts + 1):
        parts[p] = parts[p - 1] + chunk + (1 if p <= rem else 0)
    return parts


def partition_balanced(weights, num_parts, eps=1e-3):
    """Contiguous split of `weights` into num_parts minimising the heaviest part (binary search on the bound)."""
    n = len(weights)
    if n <= num_parts:
        return partition_uniform(n, num_parts)
    prefix = [0.0]
    for w in weights:
        prefix.append(prefix[-1] + w)

    def parts_for(bound):
        parts, start = [0], 0
        for _ in range(num_parts):
            end = start
            while end < n and prefix[end + 1] - prefix[start] <= bound:
                end += 1
            if end == start and start < n:
                return None
            parts.append(end)
            start = end
        return parts if parts[-1] == n else None

    lo, hi = max(weights), prefix[-1]
    best = parts_for(hi)
    while hi - lo > eps * max(hi, 1e-12):
        mid = (lo + hi) / 2
        p = parts_for(mid)
        if p is None:
            lo = mid
        else:
            best, hi = p, mid
    return best


def align_dense_tensors(tensor_list, alignment):
    num = sum(t.numel() for t in tensor_list)
    rem = num % alignment
    if rem:
        pad = alignment - rem
        tensor_list = list(tensor_list) + [torch.zeros(pad, device=tensor_list[0].device,
                                                       dtype=tensor_list[0].dtype)]
    return tensor_list


def all_gather_dp_groups(groups_flat, partitioned_param_groups, dp_process_group, start_alignment_factor=2,
                         allgather_bucket_size=None):
    for gi, flat in enumerate(groups_flat):
        shard = partitioned_param_groups[gi]
        dist.all_gather_into_tensor(flat, shard, group=dp_process_group[gi])


def see_memory_usage(message, force=False):
    if not force:
        return
    if dist.is_initialized() and dist.get_rank() != 0:
        return
    gc.collect()
    acc = get_accelerator()
    import psutil
    vm = psutil.virtual_memory()
    if acc.device_name() != "cpu":
        logger.info(f"{message} | MA {acc.memory_allocated() / 2**30:.2f} GB | Max_MA "
                    f"{acc.max_memory_allocated() / 2**30:.2f} GB | CA {acc.memory_reserved() / 2**30:.2f} GB | "
                    f"CPU used {(vm.total - vm.available) / 2**30:.2f} GB ({vm.percent}%)")
    else:
        logger.info(f"{message} | CPU used {(vm.total - vm.available) / 2**30:.2f} GB ({vm.percent}%)")
    acc.reset_peak_memory_stats() if hasattr(acc, "reset_peak_memory_stats") else None


def call_to_str(base, *args, **kwargs):
    name = f"{base}("
    name += ", ".join(repr(a) for a in args)
    if kwargs:
        name += (", " if args else "") + ", ".join(f"{k}={v!r}" for k, v in kwargs.items())
    return name + ")"


def get_only_unique_item(items):
    s = set(items)
    if len(s) != 1:
        raise RuntimeError(f"expected exactly one unique item, got {s}")
    return s.pop()


# ------------------------------------------------------------------------------------------------ small helpers
class DummyOptim:
    """Placeholder optimizer over the model's parameters when the client trains without one (reference
    `runtime/utils.py:DummyOptim`): gives ZeRO a param_groups list to partition."""

    def __init__(self, params):
        self.param_groups = [{"params": list(params)}]


class noop_context:
    """`with noop_context():` does nothing (stands in for optional contexts)."""

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def required_torch_version(min_version=None, max_version=None):
    from packaging import version as V
    cur = V.parse(torch.__version__.split("+")[0])
    if min_version is not None and cur < V.parse(str(min_version)):
        return False
    if max_version is not None and cur > V.parse(str(max_version)):
        return False
    return True


def bwc_tensor_model_parallel_rank(mpu=None):
    """Tensor-model-parallel rank from whichever accessor the client's `mpu` has (old and new Megatron names)."""
    if mpu is None:
        return 0
    for name in ("get_tensor_model_parallel_rank", "get_slice_parallel_rank", "get_model_parallel_rank"):
        if hasattr(mpu, name):
            return getattr(mpu, name)()
    return 0


def move_to_device(item, device, criterion_func=None):
    """Move every tensor inside a nested list / tuple / dict (for which `criterion_func` holds) to `device`."""
    ok = criterion_func or (lambda t: True)
    if torch.is_tensor(item):
        return item.to(device) if ok(item) else item
    if isinstance(item, (list, tuple)):
        return type(item)(move_to_device(v, device, criterion_func) for v in item)
    if isinstance(item, dict):
        return {k: move_to_device(v, device, criterion_func) for k, v in item.items()}
    return item


def copy_to_device(item, device, criterion_func=None):
    """As `move_to_device` but always a fresh copy (the source keeps its storage)."""
    ok = criterion_func or (lambda t: True)
    if torch.is_tensor(item):
        return item.detach().clone().to(device) if ok(item) else item
    if isinstance(item, (list, tuple)):
        return type(item)(copy_to_device(v, device, criterion_func) for v in item)
    if isinstance(item, dict):
        return {k: copy_to_device(v, device, criterion_func) for k, v in item.items()}
    return item


def get_global_norm(norm_list):
    """2-norm of a list of 2-norms."""
    return float(sum(float(n)**2 for n in norm_list))**0.5


def clip_tensors_by_global_norm(input_tensors, max_norm=1.0, global_norm=None, mpu=None, eps=1e-6, use_graph=False):
    """Scale the tensors in place so their joint 2-norm is at most `max_norm`; returns the norm before clipping."""
    if global_norm is None:
        global_norm = get_global_norm_of_tensors(input_tensors, mpu=mpu, use_graph=use_graph)
    clip = float(max_norm) / (float(global_norm) + eps)
    if clip < 1.0:
        for t in input_tensors:
            t.detach().mul_(clip)
    return global_norm


def clip_gradients(parameters, max_norm=1.0, global_grad_norm=None, mpu=None, eps=1e-6):
    """Clip `.grad` of the parameters by their (given or computed) global norm; returns that norm."""
    grads = [p.grad for p in parameters if p.grad is not None]
    if global_grad_norm is None:
        global_grad_norm = get_global_norm_of_tensors(grads, mpu=mpu)
    clip = float(max_norm) / (float(global_grad_norm) + eps)
    if clip < 1.0:
        for g in grads:
            g.detach().mul_(clip)
    return global_grad_norm


def empty_cache():
    from ..accelerator import get_accelerator
    get_accelerator().empty_cache()
    get_accelerator().reset_peak_memory_stats()


def get_ma_status():
    from ..accelerator import get_accelerator
    from .. import comm as dist
    if dist.is_initialized() and dist.get_rank() != 0:
        return 0
    return get_accelerator().memory_allocated()


_mem_alloced = 0
_mem_cached = 0


def memory_status(msg, print_rank=-1, reset_max=False):
    """One line with allocated / cached device memory and their change since the last call."""
    global _mem_alloced, _mem_cached
    from ..accelerator import get_accelerator
    from .. import comm as dist
    rank = dist.get_rank() if dist.is_initialized() else 0
    if print_rank != -1 and rank != print_rank:
        return
    acc = get_accelerator()
    acc.synchronize()
    if reset_max:
        acc.reset_max_memory_cached()
        acc.reset_max_memory_allocated()
    new_a, new_c = acc.memory_allocated(), acc.memory_cached()
    da, dc = new_a - _mem_alloced, new_c - _mem_cached
    _mem_alloced, _mem_cached = new_a, new_c
    gb = 1024**3
    print(f"RANK={rank} MEMSTATS {msg} device={acc.current_device_name()} current alloc={new_a / gb:0.4f}GB "
          f"(delta={da / gb:0.4f}GB max={acc.max_memory_allocated() / gb:0.4f}GB) current cache={new_c / gb:0.4f}GB "
          f"(delta={dc / gb:0.4f}GB max={acc.max_memory_cached() / gb:0.4f}GB)")


def prefix_sum_inc(weights):
    """Inclusive prefix sum of a list."""
    out, run = [], 0
    for w in weights:
        run += w
        out.append(run)
    return out


def get_inactive_params(param_list):
    """ZeRO-3 parameters of the list that are not gathered at the moment."""
    return [p for p in param_list if getattr(p, "ds_status", None) is not None and p.numel() == 0]

