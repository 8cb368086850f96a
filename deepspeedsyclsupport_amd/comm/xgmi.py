"""Fast small-message all-reduce paths behind `comm.inference_all_reduce`.

Reference: `inference_all_reduce` (`deepspeed/comm/comm.py`, `deepspeed/comm/ccl.py`) backed by the oneCCL-op
shared-memory all-reduce (`csrc/cpu/comm/ccl.cpp:540-611`) on CPU nodes and by the backend's all-reduce elsewhere.

Here:
  * device tensors on one node -> `XgmiAllReduce`: peer-mapped buffers over xGMI (`csrc/comm/xgmi_allreduce.hip`),
    one kernel per call (one-shot up to `DS_XGMI_AR_ONESHOT_MAX` bytes, two-shot up to the buffer capacity), no host
    synchronisation, capturable in HIP graphs; larger messages go to RCCL;
  * host tensors on one node -> `ShmAllReduce`: the POSIX-shm reduce-scatter / all-gather of `csrc/cpu/shm_comm.cpp`.
Both are built lazily per process group, collectively (every rank of the group reaches the first call together, as
it does for any collective), and can be switched off with DS_XGMI_AR=0 / DS_SHM_AR=0.
"""
import os
import socket

import torch
import torch.distributed as tdist

ONESHOT_MAX = int(os.environ.get("DS_XGMI_AR_ONESHOT_MAX", str(256 << 10)))
XGMI_CAP = int(os.environ.get("DS_XGMI_AR_MAX", str(8 << 20)))
SHM_CAP = int(os.environ.get("DS_SHM_AR_MAX", str(8 << 20)))

_xgmi = {}
_shm = {}


def _group_key(group):
    return id(group) if group is not None else 0


def _same_node(group):
    names = [None] * tdist.get_world_size(group)
    tdist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


class XgmiAllReduce:
    """Per-group peer-mapped all-reduce for device tensors (one rank per GPU, all on one node)."""

    def __init__(self, group=None, cap_bytes=XGMI_CAP):
        from ..ops.native import hip_ops
        self.ext = hip_ops()
        self.group = group
        self.world = tdist.get_world_size(group)
        self.rank = tdist.get_rank(group)
        if not 2 <= self.world <= self.ext.xar_max_world():
            raise ValueError(f"xGMI all-reduce supports 2..{self.ext.xar_max_world()} ranks, got {self.world}")
        self.id = self.ext.xar_create(self.world, self.rank, cap_bytes)
        self.cap = self.ext.xar_cap(self.id)
        if os.environ.get("DS_XGMI_AR_TIMEOUT_MS"):
            self.set_timeout_ms(float(os.environ["DS_XGMI_AR_TIMEOUT_MS"]))
        handles = [None] * self.world
        tdist.all_gather_object(handles, self.ext.xar_handles(self.id), group=group)
        for p, h in enumerate(handles):
            if p != self.rank:
                self.ext.xar_open(self.id, p, h)
        tdist.barrier(group=group)  # every peer mapped before anyone pushes

    def supports(self, t):
        return t.is_cuda and t.is_contiguous() and t.dtype in (torch.bfloat16, torch.float16, torch.float32) \
            and (t.numel() * t.element_size()) % 16 == 0 and 0 < t.numel() * t.element_size() <= self.cap

    def all_reduce(self, t, out=None, mode=None):
        """Sum over the group into `out` (default: in place). mode 1 one-shot, 2 two-shot, None by size."""
        out = t if out is None else out
        if mode is None:
            mode = 1 if t.numel() * t.element_size() <= ONESHOT_MAX else 2
        self.ext.xar_allreduce(self.id, t, out, mode)
        return out

    def error(self, reset=False):
        """0 if every wait completed; 1 + peer index of a wait that timed out (sticky; synchronises). A timed-out
        call fills its output with NaN and every later `all_reduce` raises until the word is reset."""
        return self.ext.xar_error(self.id, reset)

    def set_timeout_ms(self, ms):
        """Wait limit of the in-kernel peer waits (default 5 s; DS_XGMI_AR_TIMEOUT_MS at construction)."""
        self.ext.xar_set_timeout_ms(self.id, float(ms))

    def close(self):
        if self.id is not None:
            self.ext.xar_destroy(self.id)
            self.id = None


class ShmAllReduce:
    """Per-group POSIX-shm all-reduce for host fp32/bf16 tensors (ranks of one node)."""

    def __init__(self, group=None, cap_bytes=SHM_CAP):
        from ..ops.op_builder import load
        self.ext = load("ds_cpu_ops")
        self.group = group
        ranks = tdist.get_process_group_ranks(group) if group is not None else list(range(tdist.get_world_size()))
        self.rank = tdist.get_rank(group)
        self.world = len(ranks)
        # unique per job and group: master port + the group's global ranks
        tag = f"{os.environ.get('MASTER_PORT', '0')}_{'-'.join(map(str, ranks))}"
        self.name = f"/ds_amd_shm_{os.getuid()}_{tag}"[:250]
        if self.rank == 0:
            self.handle = self.ext.shm_init(self.name, 0, self.world, cap_bytes)
        tdist.barrier(group=group)
        if self.rank != 0:
            self.handle = self.ext.shm_init(self.name, self.rank, self.world, cap_bytes)
        tdist.barrier(group=group)
        if self.rank == 0:
            self.ext.shm_release_name(self.handle)

    def supports(self, t):
        return (not t.is_cuda) and t.is_contiguous() and t.dtype in (torch.float32, torch.bfloat16)

    def all_reduce(self, t):
        self.ext.shm_allreduce(self.handle, t)
        return t

    def close(self):
        if self.handle is not None:
            self.ext.shm_finalize(self.handle)
            self.handle = None


def _xgmi_for(group):
    key = _group_key(group)
    if key not in _xgmi:
        ok = os.environ.get("DS_XGMI_AR", "1") != "0" and tdist.get_backend(group) == "nccl" and \
            2 <= tdist.get_world_size(group) <= 8 and _same_node(group)
        _xgmi[key] = XgmiAllReduce(group) if ok else None
    return _xgmi[key]


def _shm_for(group):
    key = _group_key(group)
    if key not in _shm:
        ok = os.environ.get("DS_SHM_AR", "1") != "0" and tdist.get_world_size(group) > 1 and _same_node(group)
        _shm[key] = ShmAllReduce(group) if ok else None
    return _shm[key]


def fast_all_reduce(tensor, group=None):
    """Sum all-reduce through the fast path if one applies; returns True if it handled the tensor."""
    if tdist.get_world_size(group) == 1:
        return True
    if tensor.is_cuda:
        xa = _xgmi_for(group)
        if xa is not None and xa.supports(tensor):
            xa.all_reduce(tensor)
            return True
        return False
    sa = _shm_for(group)
    if sa is not None and sa.supports(tensor):
        sa.all_reduce(tensor)
        return True
    return False


def reset():
    """Tear down cached communicators (tests / re-initialisation)."""
    for c in list(_xgmi.values()) + list(_shm.values()):
        if c is not None:
            c.close()
    _xgmi.clear()
    _shm.clear()
