"""Process groups of MiCS (reference `runtime/zero/mics_utils.py`): the data-parallel ranks are cut into shard groups
of `shard_size` consecutive ranks that partition the model states among themselves, and replica groups (one rank of
every shard group) that all-reduce gradients between the copies. A shard group wider than a node also gets the two
groups of the hierarchical parameter gather: the ranks of one node inside it, and the ranks of one local index
across its nodes."""
import os
from dataclasses import dataclass
from typing import Any

from ... import comm as dist
from ...accelerator import get_accelerator


@dataclass
class MiCS_CommGroups:
    param_shard_group: Any = None
    param_shard_size: int = -1
    param_shard_rank: int = -1
    param_repli_group: Any = None
    param_repli_size: int = -1
    param_repli_rank: int = -1
    param_intra_node_group: Any = None
    param_inter_node_shard_group: Any = None


def scale_tensors(tensors, scale):
    """Divide every tensor in place by `scale`."""
    for t in tensors:
        t.div_(scale)


def node_size():
    """GPUs per node: `DS_NODE_SIZE` when set (tests, irregular machines), else the local device count."""
    return int(os.environ.get("DS_NODE_SIZE", 0)) or max(get_accelerator().device_count(), 1)


def create_mics_comm_groups(shard_size, dp_group=None, hierarchical_allgather=False, mpu=None, ranks=None):
    """Every rank of `dp_group` must call this (group creation is collective). `ranks`: the group's global ranks
    when the caller already knows them."""
    if ranks is None:
        ranks = dist.get_all_ranks_from_group(dp_group) if dp_group is not None else \
            list(range(dist.get_world_size()))
    dp = len(ranks)
    if dp % shard_size:
        raise ValueError(f"mics_shard_size {shard_size} must divide the data-parallel size {dp}")
    me = dist.get_rank()
    out = MiCS_CommGroups(param_shard_size=shard_size, param_repli_size=dp // shard_size)
    for i in range(dp // shard_size):
        grp = ranks[i * shard_size:(i + 1) * shard_size]
        g = dist.new_group(grp)
        if me in grp:
            out.param_shard_group, out.param_shard_rank = g, grp.index(me)
    for j in range(shard_size):
        grp = ranks[j::shard_size]
        g = dist.new_group(grp)
        if me in grp:
            out.param_repli_group, out.param_repli_rank = g, grp.index(me)
    node = node_size()
    if hierarchical_allgather and shard_size > node and shard_size % node == 0:
        for i in range(dp // shard_size):
            grp = ranks[i * shard_size:(i + 1) * shard_size]
            for a in range(shard_size // node):       # the ranks of one node inside this shard group
                sub = grp[a * node:(a + 1) * node]
                g = dist.new_group(sub)
                if me in sub:
                    out.param_intra_node_group = g
            for b in range(node):                     # one local index across the shard group's nodes
                sub = grp[b::node]
                g = dist.new_group(sub)
                if me in sub:
                    out.param_inter_node_shard_group = g
    return out
