"""Cross-rank consistency checks — the framework's race / divergence detector (reference `runtime/zero/utils.py:60-89`
`assert_ints_same_as_other_ranks`, the ZeRO-3 all-gather / reduce `safe_mode` checks of `partition_parameters.py:1139`
and `stage3.py:1205`, and the trace validation of `partitioned_param_coordinator.py:200-216`).

Collectives deadlock or silently mix unrelated buffers when ranks issue them in different orders (a data-dependent
branch, an unused parameter on one rank, a module called twice). With `zero_optimization.safe_mode: true` every
ZeRO collective is preceded by a tiny all-reduce that proves all ranks are about to run the SAME collective on the
SAME buffer (fetch-group id + element count), every step's fetch trace is compared across ranks, and a group
reduced twice in one backward pass raises. The checks cost a host sync each, so they are a debug mode.
"""
import hashlib

import torch

from ... import comm as dist


class ZeRORuntimeException(RuntimeError):
    pass


def _device_for(group):
    try:
        backend = dist.get_backend(group)
    except Exception:  # noqa: BLE001
        backend = "gloo"
    if str(backend).lower() in ("nccl", "rccl") and torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def assert_ints_same_as_other_ranks(ints, group=None, what="values"):
    """Raise ZeRORuntimeException unless every rank of `group` passes the same list of ints (as rank 0 does).

    Implemented as min/max all-reduces (two collectives, one tensor each) so a mismatch is detected on EVERY rank,
    not just the ones that differ from rank 0 — all ranks then raise together instead of some hanging."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dev = _device_for(group)
    t = torch.tensor([len(ints)] + [int(i) for i in ints], dtype=torch.int64, device=dev)
    lo, hi = t.clone(), t.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    if not torch.equal(lo, hi):
        raise ZeRORuntimeException(f"rank {dist.get_rank()}: {what} differ across ranks: mine={list(ints)} "
                                   f"min={lo.tolist()[1:]} max={hi.tolist()[1:]}")


def trace_digest(trace):
    """64-bit digest of a fetch trace (list of group ids) for cheap cross-rank comparison."""
    h = hashlib.sha1(",".join(map(str, trace)).encode()).digest()
    return [len(trace), int.from_bytes(h[:7], "little")]


def _zero_supported_optimizers():
    import torch
    from ...ops.adagrad.cpu_adagrad import DeepSpeedCPUAdagrad
    from ...ops.adam.cpu_adam import DeepSpeedCPUAdam
    from ...ops.adam.fused_adam import FusedAdam
    out = [torch.optim.Adam, torch.optim.AdamW, FusedAdam, DeepSpeedCPUAdam, torch.optim.Adagrad,
           DeepSpeedCPUAdagrad]
    try:
        from ...ops.lion.fused_lion import FusedLion
        from ...ops.lion.cpu_lion import DeepSpeedCPULion
        out += [FusedLion, DeepSpeedCPULion]
    except ImportError:
        pass
    return out


def is_zero_supported_optimizer(optimizer):
    """Is the optimizer one of those tested under ZeRO? (others need `zero_allow_untested_optimizer`)"""
    return type(optimizer) in _zero_supported_optimizers()


def get_lst_from_rank0(lst):
    """Broadcast a list of ints from rank 0; every rank gets rank 0's values."""
    import torch
    from ... import comm as dist
    t = torch.tensor(lst if dist.get_rank() == 0 else [-1] * len(lst), dtype=torch.int64,
                     device=_device_for(None))
    dist.broadcast(t, src=0)
    return t.cpu().tolist()

