"""Process-group registry: DP, sequence(SP)×DP, expert (EP) / expert-data, TP (via mpu), hpZ and the local/global
all-to-all groups used by qgZ.

Reference: `deepspeed/utils/groups.py:64-562` (same accessor names, same rank layouts). MI355X-first choice: SP,
TP, EP and hpZ groups are built from CONSECUTIVE ranks so that on an 8-GPU node they stay inside one xGMI full
mesh (every peer pair has its own ≈153 GB/s link, ideal for all-to-all); DP (and the sequence×data ZeRO group)
spans the rest.
"""
import torch

from .. import comm as dist
from ..accelerator import get_accelerator
from ..utils.logging import log_dist

_EXPERT_PARALLEL_GROUP = {}
_EXPERT_DATA_PARALLEL_GROUP = {}
_WORLD_GROUP = None
_ZERO_PARAM_INTRA_PARALLEL_GROUP = None
_DATA_PARALLEL_GROUP = None
_SEQUENCE_PARALLEL_GROUP = None
_SEQUENCE_DATA_PARALLEL_GROUP = None
_SP_SIZE = 1
_ALL_TO_ALL_GROUP = {}
mpu = None
expert_tensor_parallel_world_size = 1


def _ensure_divisibility(numerator, denominator):
    assert numerator % denominator == 0, f"{numerator} is not divisible by {denominator}"


def reset():
    """Forget every group (tests create several engines per process)."""
    global _EXPERT_PARALLEL_GROUP, _EXPERT_DATA_PARALLEL_GROUP, _WORLD_GROUP, _ZERO_PARAM_INTRA_PARALLEL_GROUP
    global _DATA_PARALLEL_GROUP, _SEQUENCE_PARALLEL_GROUP, _SEQUENCE_DATA_PARALLEL_GROUP, _SP_SIZE, mpu
    global _ALL_TO_ALL_GROUP
    _EXPERT_PARALLEL_GROUP, _EXPERT_DATA_PARALLEL_GROUP, _ALL_TO_ALL_GROUP = {}, {}, {}
    _WORLD_GROUP = _ZERO_PARAM_INTRA_PARALLEL_GROUP = _DATA_PARALLEL_GROUP = None
    _SEQUENCE_PARALLEL_GROUP = _SEQUENCE_DATA_PARALLEL_GROUP = None
    _SP_SIZE = 1
    mpu = None
    global expert_tensor_parallel_world_size
    expert_tensor_parallel_world_size = 1


# ------------------------------------------------------------------------------------------- model parallel
def initialize(ep_size=1, mpu_=None):
    """Deprecated entry kept for parity (`groups.py:48`)."""
    global mpu
    if mpu_ is not None:
        mpu = mpu_
    if ep_size > 1:
        _create_expert_and_data_parallel(ep_size)


def _create_model_parallel(model_parallel_size_):
    """DP and MP groups over consecutive-rank MP blocks (`groups.py:64-110`)."""
    world_size = dist.get_world_size()
    rank = dist.get_rank()
    _ensure_divisibility(world_size, model_parallel_size_)
    dp_group = mp_group = None
    for i in range(model_parallel_size_):
        ranks = list(range(i, world_size, model_parallel_size_))
        g = dist.new_group(ranks)
        if i == rank % model_parallel_size_:
            dp_group = g
    for i in range(world_size // model_parallel_size_):
        ranks = list(range(i * model_parallel_size_, (i + 1) * model_parallel_size_))
        g = dist.new_group(ranks)
        if i == rank // model_parallel_size_:
            mp_group = g
    return dp_group, mp_group


# ------------------------------------------------------------------------------------------- sequence parallel
def initialize_sequence_parallel(sp_size):
    """Build Ulysses SP groups (consecutive ranks → one xGMI mesh) and the sequence×data ZeRO group (= world).

    Used when the user passes no `mpu`; equivalent to the mpu Megatron-DeepSpeed provides to the reference
    (`groups.py:452-497`).
    """
    global _SEQUENCE_PARALLEL_GROUP, _SEQUENCE_DATA_PARALLEL_GROUP, _DATA_PARALLEL_GROUP, _SP_SIZE
    world = dist.get_world_size()
    rank = dist.get_rank()
    _ensure_divisibility(world, sp_size)
    _SP_SIZE = sp_size
    for i in range(world // sp_size):
        ranks = list(range(i * sp_size, (i + 1) * sp_size))
        g = dist.new_group(ranks)
        if rank in ranks:
            _SEQUENCE_PARALLEL_GROUP = g
    for i in range(sp_size):
        ranks = list(range(i, world, sp_size))
        g = dist.new_group(ranks)
        if rank in ranks:
            _DATA_PARALLEL_GROUP = g
    _SEQUENCE_DATA_PARALLEL_GROUP = _clone_world_group()
    log_dist(f"Ulysses sequence parallel: sp_size={sp_size}, dp_size={world // sp_size}", ranks=[0])


def _get_sequence_parallel_group():
    if mpu is not None and hasattr(mpu, "get_sequence_parallel_group"):
        return mpu.get_sequence_parallel_group()
    return _SEQUENCE_PARALLEL_GROUP


def _get_sequence_parallel_world_size():
    if mpu is not None and hasattr(mpu, "get_sequence_parallel_world_size"):
        return mpu.get_sequence_parallel_world_size()
    return _SP_SIZE


def _get_sequence_parallel_rank():
    if mpu is not None and hasattr(mpu, "get_sequence_parallel_rank"):
        return mpu.get_sequence_parallel_rank()
    g = _SEQUENCE_PARALLEL_GROUP
    return dist.get_rank(g) if g is not None else 0


def _get_sequence_data_parallel_group():
    if mpu is not None and hasattr(mpu, "get_sequence_data_parallel_group"):
        return mpu.get_sequence_data_parallel_group()
    if _SEQUENCE_DATA_PARALLEL_GROUP is not None:
        return _SEQUENCE_DATA_PARALLEL_GROUP
    return _get_data_parallel_group()


def _get_sequence_data_parallel_world_size():
    if mpu is not None and hasattr(mpu, "get_sequence_data_parallel_world_size"):
        return mpu.get_sequence_data_parallel_world_size()
    return dist.get_world_size(_get_sequence_data_parallel_group())


def _get_sequence_data_parallel_rank():
    if mpu is not None and hasattr(mpu, "get_sequence_data_parallel_rank"):
        return mpu.get_sequence_data_parallel_rank()
    return dist.get_rank(_get_sequence_data_parallel_group())


# ------------------------------------------------------------------------------------------- expert parallel
def _create_expert_and_data_parallel(expert_parallel_size_, use_data_before_expert_parallel_=False):
    """E+D (default) or D+E layouts exactly as `groups.py:113-177`; E+D keeps each EP group on consecutive ranks."""
    world_size = dist.get_world_size()
    rank = dist.get_rank()
    _ensure_divisibility(world_size, expert_parallel_size_)
    name = f"ep_size_{expert_parallel_size_}"
    ep_stride = world_size // expert_parallel_size_
    if name not in _EXPERT_DATA_PARALLEL_GROUP:
        for i in range(expert_parallel_size_):
            ranks = list(range(i * ep_stride, (i + 1) * ep_stride)) if use_data_before_expert_parallel_ \
                else list(range(i, world_size, expert_parallel_size_))
            g = dist.new_group(ranks)
            if rank in ranks:
                _EXPERT_DATA_PARALLEL_GROUP[name] = g
    if name not in _EXPERT_PARALLEL_GROUP:
        if use_data_before_expert_parallel_:
            for i in range(ep_stride):
                ranks = list(range(i, world_size, ep_stride))
                g = dist.new_group(ranks)
                if rank in ranks:
                    _EXPERT_PARALLEL_GROUP[name] = g
        else:
            for i in range(world_size // expert_parallel_size_):
                ranks = list(range(i * expert_parallel_size_, (i + 1) * expert_parallel_size_))
                g = dist.new_group(ranks)
                if rank in ranks:
                    _EXPERT_PARALLEL_GROUP[name] = g


def _get_expert_parallel_ranks(world_size, model_parallel_size_, expert_parallel_size_,
                               use_data_before_expert_parallel_=False):
    """Rank lists of the expert-parallel and expert-data-parallel groups under tensor (model) parallelism (reference
    `groups.py:179-236`). Model-parallel groups are blocks of consecutive ranks; the ranks with the same position in
    their block form one data-parallel line, and every line is cut into expert-parallel groups of
    `expert_parallel_size_` members (E+D), or strided so that data-parallel neighbours stay adjacent (D+E). E.g.
    world 16, model 2, expert 4: EP [0,2,4,6] [8,10,12,14] [1,3,5,7] [9,11,13,15]; EDP [0,8] [2,10] ... [7,15]."""
    _ensure_divisibility(world_size, model_parallel_size_)
    dp_world = world_size // model_parallel_size_
    _ensure_divisibility(dp_world, expert_parallel_size_)
    lines = []
    for i in range(model_parallel_size_):
        if use_data_before_expert_parallel_:
            stride = dp_world // expert_parallel_size_
            line = []
            for d in range(stride):
                line += list(range(i + d * model_parallel_size_, world_size, stride * model_parallel_size_))
            lines.append(line)
        else:
            lines.append(list(range(i, world_size, model_parallel_size_)))
    ep_groups, edp_groups = [], []
    for line in lines:
        parts = [line[i:i + expert_parallel_size_] for i in range(0, dp_world, expert_parallel_size_)]
        ep_groups += parts
        edp_groups += [list(t) for t in zip(*parts)]
    return ep_groups, edp_groups


def _create_expert_data_and_model_parallel(expert_parallel_size_, mpu, use_data_before_expert_parallel_=False):
    """Expert groups for experts that ARE tensor parallel (reference `groups.py:239-290`): built inside each
    data-parallel line of the mpu, and the expert tensor-parallel degree is recorded so the MoE layer keeps the
    duplicated tokens (every TP rank of an expert needs them)."""
    global expert_tensor_parallel_world_size
    mp = mpu.get_model_parallel_world_size()
    expert_tensor_parallel_world_size = mp
    world_size, rank = dist.get_world_size(), dist.get_rank()
    name = f"ep_size_{expert_parallel_size_}"
    log_dist(f"Creating expert groups with model parallel size {mp}, expert parallel size {expert_parallel_size_}, "
             f"world size {world_size}", ranks=[0])
    if name in _EXPERT_DATA_PARALLEL_GROUP or name in _EXPERT_PARALLEL_GROUP:
        return
    ep_groups, edp_groups = _get_expert_parallel_ranks(world_size, mp, expert_parallel_size_,
                                                       use_data_before_expert_parallel_)
    for ranks in ep_groups:
        g = dist.new_group(ranks)
        if rank in ranks:
            _EXPERT_PARALLEL_GROUP[name] = g
    for ranks in edp_groups:
        g = dist.new_group(ranks)
        if rank in ranks:
            _EXPERT_DATA_PARALLEL_GROUP[name] = g


def _get_max_expert_size():
    sizes = [int(k.split("_")[-1]) for k in _EXPERT_PARALLEL_GROUP]
    return max(sizes) if sizes else None


def _get_max_expert_size_name():
    return f"ep_size_{_get_max_expert_size()}"


def _get_max_expert_parallel_group():
    return _get_expert_parallel_group(_get_max_expert_size_name())


def _get_expert_parallel_group(group_name):
    assert group_name in _EXPERT_PARALLEL_GROUP, "expert parallel group is not initialized"
    return _EXPERT_PARALLEL_GROUP[group_name]


def _get_expert_parallel_group_dict():
    return _EXPERT_PARALLEL_GROUP


def _get_expert_data_parallel_group(group_name):
    assert group_name in _EXPERT_DATA_PARALLEL_GROUP, "expert data parallel group is not initialized"
    return _EXPERT_DATA_PARALLEL_GROUP[group_name]


def _get_expert_data_parallel_group_dict():
    return _EXPERT_DATA_PARALLEL_GROUP


def _get_expert_parallel_world_size(group_name):
    return dist.get_world_size(group=_get_expert_parallel_group(group_name))


def _get_expert_data_parallel_world_size(group_name):
    return dist.get_world_size(group=_get_expert_data_parallel_group(group_name))


def _get_expert_parallel_rank(group_name):
    return dist.get_rank(group=_get_expert_parallel_group(group_name))


def _get_expert_data_parallel_rank(group_name):
    return dist.get_rank(group=_get_expert_data_parallel_group(group_name))


def _get_expert_broadcast_src_rank(group_name):
    return dist.get_global_rank(_get_expert_data_parallel_group(group_name), 0)


def _get_expert_model_parallel_world_size():
    return expert_tensor_parallel_world_size


# ------------------------------------------------------------------------------------------- data parallel
def _clone_world_group():
    global _WORLD_GROUP
    if _WORLD_GROUP is None:
        _WORLD_GROUP = dist.new_group(ranks=range(dist.get_world_size())) if dist.is_initialized() else None
    return _WORLD_GROUP


def _get_data_parallel_group():
    if mpu is not None:
        return mpu.get_data_parallel_group()
    if _DATA_PARALLEL_GROUP is not None:
        return _DATA_PARALLEL_GROUP
    return _clone_world_group()


def _get_broadcast_src_rank():
    return dist.get_global_rank(_get_sequence_data_parallel_group(), 0)


def _get_data_parallel_world_size():
    if mpu is not None:
        return mpu.get_data_parallel_world_size()
    return dist.get_world_size(group=_get_data_parallel_group())


def _get_data_parallel_rank():
    if mpu is not None:
        return mpu.get_data_parallel_rank()
    return dist.get_rank(group=_get_data_parallel_group())


def _get_model_parallel_world_size():
    if mpu is not None:
        return mpu.get_model_parallel_world_size()
    return 1


def _get_model_parallel_rank():
    if mpu is not None:
        return mpu.get_model_parallel_rank()
    return 0


def _get_model_parallel_group():
    if mpu is not None:
        return mpu.get_model_parallel_group()
    return None


# ------------------------------------------------------------------------------------------- hpZ / qgZ
def _create_zero_param_parallel_group(group_size):
    """hpZ secondary-partition groups of consecutive ranks (`groups.py:505-533`)."""
    global _ZERO_PARAM_INTRA_PARALLEL_GROUP
    world_size = dist.get_world_size()
    rank = dist.get_rank()
    size = min(group_size, world_size)
    _ensure_divisibility(world_size, size)
    for i in range(world_size // size):
        ranks = list(range(i * size, (i + 1) * size))
        g = dist.new_group(ranks)
        if rank in ranks:
            _ZERO_PARAM_INTRA_PARALLEL_GROUP = g


def _get_zero_param_intra_parallel_group():
    return _ZERO_PARAM_INTRA_PARALLEL_GROUP


def _zero_param_parallel_is_initialized():
    return _ZERO_PARAM_INTRA_PARALLEL_GROUP is not None


def _get_zero_param_intra_parallel_rank_in_mygroup():
    return dist.get_rank(group=_get_zero_param_intra_parallel_group())


def _get_zero_param_intra_parallel_group_world_size():
    return dist.get_world_size(group=_get_zero_param_intra_parallel_group())


def _get_zero_param_intra_parallel_group_ranks():
    return dist.get_all_ranks_from_group(group=_get_zero_param_intra_parallel_group())


def _get_local_all_to_all_group(devices_per_node=None):
    """`local_i` (intra-node, xGMI mesh) and `global_i` (same local rank across nodes) groups (`groups.py:356-382`)."""
    global _ALL_TO_ALL_GROUP
    if _ALL_TO_ALL_GROUP:
        return _ALL_TO_ALL_GROUP
    dpn = devices_per_node or max(get_accelerator().device_count(), 1)
    world = dist.get_world_size()
    dpn = min(dpn, world)
    num_nodes = world // dpn
    for i in range(num_nodes):
        _ALL_TO_ALL_GROUP[f"local_{i}"] = dist.new_group(ranks=[j + dpn * i for j in range(dpn)])
    if num_nodes > 1:
        for i in range(dpn):
            _ALL_TO_ALL_GROUP[f"global_{i}"] = dist.new_group(ranks=[i + j * dpn for j in range(num_nodes)])
    return _ALL_TO_ALL_GROUP


def is_initialized():
    return dist.is_initialized()
