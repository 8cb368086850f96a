"""Point-to-point transfers between pipeline stages (reference `runtime/pipe/p2p.py`).

Stages exchange tensors with RCCL send / recv on the current HIP stream (`comm.send` / `comm.recv`; over xGMI when
the stages share a node); Python objects go as a length-prefixed pickled byte tensor. `init_process_groups` records
the grid so stage ids can be turned into global ranks.
"""
import pickle

import torch

from ... import comm as dist
from ...accelerator import get_accelerator

_grid = None
_async = []


def can_send_recv() -> bool:
    return True


def init_process_groups(grid):
    global _grid
    _grid = grid
    if grid.pipe_parallel_size < 2:
        raise AssertionError("pipeline p2p needs at least two stages")


def _is_valid_send_recv(src_stage, dest_stage):
    first, last = 0, _grid.pipe_parallel_size - 1
    ok = abs(src_stage - dest_stage) == 1 or (src_stage, dest_stage) in ((first, last), (last, first))
    assert ok, "Functionality currently limited to send and receive between adjacent ranks only"


def send(tensor, dest_stage, async_op=False):
    src_stage = _grid.get_stage_id()
    _is_valid_send_recv(src_stage, dest_stage)
    dest = _grid.stage_to_global(stage_id=dest_stage)
    if async_op:
        op = dist.isend(tensor, dest)
        _async.append(op)
        return op
    return dist.send(tensor, dest)


def recv(tensor, src_stage, async_op=False):
    dest_stage = _grid.get_stage_id()
    _is_valid_send_recv(src_stage, dest_stage)
    src = _grid.stage_to_global(stage_id=src_stage)
    if async_op:
        op = dist.irecv(tensor, src)
        _async.append(op)
        return op
    return dist.recv(tensor, src)


def wait():
    for op in _async:
        op.wait()
    _async.clear()
    get_accelerator().synchronize()


def _device():
    acc = get_accelerator()
    return torch.device("cpu") if dist.get_backend() == "gloo" or acc.device_name() == "cpu" else \
        torch.device(acc.device_name(acc.current_device()))


def send_obj(msg, dest: int):
    """Send a picklable object to global rank `dest`."""
    data = torch.frombuffer(bytearray(pickle.dumps(msg)), dtype=torch.uint8).to(_device())
    dist.send(torch.tensor([data.numel()], dtype=torch.long, device=data.device), dest)
    dist.send(data, dest)


def recv_obj(sender: int):
    """Receive an object sent with `send_obj` from global rank `sender` (tensors inside arrive on this device)."""
    dev = _device()
    n = torch.zeros(1, dtype=torch.long, device=dev)
    dist.recv(n, sender)
    data = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    dist.recv(data, sender)
    msg = pickle.loads(data.cpu().numpy().tobytes())

    def to_dev(x):
        if torch.is_tensor(x):
            return x.to(dev)
        if isinstance(x, (list, tuple)):
            return type(x)(to_dev(y) for y in x)
        if isinstance(x, dict):
            return {k: to_dev(v) for k, v in x.items()}
        return x

    return to_dev(msg)
