"""Host-tensor backend (reference `comm/ccl.py:34` `CCLBackend`: oneCCL plus a POSIX-shm all-reduce for single-node
inference). On this platform host tensors travel over gloo and the single-node low-latency all-reduce is the shm
reduce of `ops/csrc/cpu/shm_comm.cpp` (reached through `comm.inference_all_reduce`); this object exposes both
behind the reference's backend interface."""
import torch

from . import comm as dist
from .backend import Backend
from .reduce_op import ReduceOp


def build_ccl_op():
    """The native host extension (shm all-reduce lives in it), or None when it cannot be loaded."""
    try:
        from ..ops.native import cpu_ops
        return cpu_ops()
    except Exception:
        return None


class CCLHandler:

    def __init__(self, ccl_comm_op=None):
        self.ccl_comm_op = ccl_comm_op

    def wait(self):
        return None


class CCLBackend(Backend):

    def __init__(self, name="ccl", rank=-1, world_size=-1, mpu=None, timeout=None, init_method=None):
        super().__init__(name, rank, world_size)
        self.ccl_comm_op = build_ccl_op()
        if not dist.is_initialized():
            dist.init_distributed("gloo", timeout=timeout, init_method=init_method, rank=rank,
                                  world_size=world_size)
        self.world_rank, self.world_size = dist.get_rank(), dist.get_world_size()
        self.initialized = True
        self.groups = [tuple(range(self.world_size))]
        self.available_coll = ["broadcast", "all_reduce", "inference_all_reduce", "all_reduce_caching", "barrier"]

    def is_initialized(self):
        return self.initialized

    def get_all_ranks_from_group(self, group):
        return list(range(dist.get_world_size(group)))

    def all_reduce(self, tensor, op=ReduceOp.SUM, group=None, async_op=False):
        return dist.all_reduce(tensor, op=op, group=group, async_op=async_op)

    def inference_all_reduce(self, tensor, op=ReduceOp.SUM, group=None, async_op=False):
        return dist.inference_all_reduce(tensor, op=op, group=group, async_op=async_op)

    def all_reduce_caching(self, tensor, op=ReduceOp.SUM, match_id=None, group=None, async_op=False):
        return dist.all_reduce(tensor, op=op, group=group, async_op=async_op)

    def broadcast(self, tensor, src, group=None, async_op=False):
        return dist.broadcast(tensor, src, group=group, async_op=async_op)

    def barrier(self, group=None, async_op=False):
        return dist.barrier(group=group)

    def all_gather(self, tensor_list, tensor, group=None, async_op=False):
        return dist.all_gather(tensor_list, tensor, group=group, async_op=async_op)

    def reduce_scatter_tensor(self, output_tensor, input_tensor, op=ReduceOp.SUM, group=None, async_op=False):
        return dist.reduce_scatter_tensor(output_tensor, input_tensor, op=op, group=group, async_op=async_op)

    def all_gather_into_tensor(self, output_tensor, input_tensor, group=None, async_op=False):
        return dist.all_gather_into_tensor(output_tensor, input_tensor, group=group, async_op=async_op)


_ = torch
