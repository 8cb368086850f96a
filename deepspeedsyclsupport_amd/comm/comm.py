"""`deepspeedsyclsupport_amd.comm`: torch.distributed-compatible collective facade over RCCL (xGMI) / gloo.

Reference: `deepspeed/comm/comm.py:222-604` (facade + `timed_op` + `init_distributed`) and
`deepspeed/comm/torch.py:99-151` (TorchBackend). The reference routes through a global backend object so it
can swap in oneCCL; on MI355X there is one backend — torch.distributed with `nccl` (= RCCL on ROCm) for device
tensors and `gloo` on the host path — so this module calls torch.distributed directly and only adds:
  * `timed_op` comms logging (algbw/busbw + per-xGMI-link figure),
  * process-group bookkeeping for `get_world_group`, `new_group`,
  * `inference_all_reduce` over the native small-message paths of `comm/xgmi.py` (xGMI peer-mapped kernel for
    device tensors, POSIX shm for host tensors).
The ZeRO bucketed collectives (the reference's `runtime/comm/coalesced_collectives.py`) are issued directly by the
flat-group optimizer (`runtime/zero/flat_optimizer.py`, `runtime/zero/zeropp.py`).
"""
import functools
import os
import socket
import time
from datetime import timedelta

import torch
import torch.distributed as tdist

from ..accelerator import get_accelerator
from ..utils.logging import logger
from .comms_logging import CommsLogger
from .reduce_op import ReduceOp

default_pg_timeout = timedelta(minutes=int(os.environ.get("DS_PG_TIMEOUT_MIN", "30")))
TORCH_DISTRIBUTED_DEFAULT_PORT = 29500

comms_logger = CommsLogger()
timers_enabled = False
prof_all = False
debug = False


class ProcessGroup:
    """Placeholder kept for API parity (`deepspeed/comm/comm.py:33`)."""

    def __init__(self, comm_id, ranks=None):
        self.ranks = ranks or []
        self.comm_id = comm_id
        self.size = len(self.ranks)


def configure(deepspeed_config=None, enabled=None, prof_all=None, prof_ops=None, verbose=None, debug=None):
    if deepspeed_config is not None:
        comms_logger.configure(deepspeed_config.comms_config)
    if enabled is not None:
        comms_logger.enabled = enabled
    if prof_all is not None:
        comms_logger.prof_all = prof_all
    if prof_ops is not None:
        comms_logger.prof_ops = prof_ops
    if verbose is not None:
        comms_logger.verbose = verbose
    if debug is not None:
        comms_logger.debug = debug


def _msg_size(name, args, kwargs):
    for t in list(args) + list(kwargs.values()):
        if torch.is_tensor(t):
            return t.numel() * t.element_size()
        if isinstance(t, (list, tuple)) and t and torch.is_tensor(t[0]):
            return sum(x.numel() * x.element_size() for x in t)
    return 0


def timed_op(func):
    """Time the collective when the comms logger is on (synchronizes the device; debugging aid only)."""

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        if not comms_logger.enabled:
            return func(*args, **kwargs)
        log_name = kwargs.pop("log_name", func.__name__)
        if not (comms_logger.prof_all or log_name in comms_logger.prof_ops):
            return func(*args, **kwargs)
        acc = get_accelerator()
        acc.synchronize()
        t0 = time.perf_counter()
        out = func(*args, **kwargs)
        if kwargs.get("async_op") and out is not None:
            out.wait()
        acc.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        grp = kwargs.get("group")
        comms_logger.append(func.__name__, log_name, dt, _msg_size(func.__name__, args, kwargs), get_world_size(grp))
        return out

    return wrapper


# ---------------------------------------------------------------------------------------------- init
def is_initialized():
    return tdist.is_available() and tdist.is_initialized()


def is_available():
    return tdist.is_available()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def init_distributed(dist_backend=None, auto_mpi_discovery=True, distributed_port=TORCH_DISTRIBUTED_DEFAULT_PORT,
                     verbose=True, timeout=default_pg_timeout, init_method=None, dist_init_required=None, config=None,
                     rank=-1, world_size=-1):
    """Initialise torch.distributed (RCCL on MI355X, gloo on the host path).

    Env contract as in the reference (`comm.py:604-670`): RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT/LOCAL_RANK.
    Without them we fall back to MPI discovery (OMPI_/PMI_ env vars) and finally to a single-process group on
    127.0.0.1 so scripts run unchanged on one GPU.
    """
    if config is not None:
        configure(deepspeed_config=config)
    if is_initialized():
        return
    if dist_init_required is False:
        return
    if dist_backend is None:
        dist_backend = get_accelerator().communication_backend_name()
    required = ["RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
    if not all(k in os.environ for k in required):
        if in_aml() and not in_dlts():
            patch_aml_env_for_torch_nccl_backend(master_port=distributed_port, verbose=verbose)
        elif in_aws_sm():
            patch_aws_sm_env_for_torch_nccl_backend(verbose=verbose)
    if not all(k in os.environ for k in required):
        if auto_mpi_discovery and _mpi_env_discovery(distributed_port, verbose):
            pass
        elif rank < 0:
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("LOCAL_RANK", "0")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("LOCAL_RANK", os.environ.get("RANK", "0"))
    if dist_backend == "nccl":
        local_rank = int(os.environ["LOCAL_RANK"])
        get_accelerator().set_device(local_rank % max(get_accelerator().device_count(), 1))
    kw = dict(backend=dist_backend, timeout=timeout)
    if init_method is not None:
        kw["init_method"] = init_method
    if rank >= 0:
        kw["rank"] = rank
        kw["world_size"] = world_size
    if dist_backend == "nccl":
        # bind the PG to our device up front: lets RCCL create communicators eagerly and avoids the
        # "guessing device" barrier path
        kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    if verbose and int(os.environ.get("RANK", "0")) == 0:
        logger.info(f"Initializing torch.distributed with backend {dist_backend}")
    tdist.init_process_group(**kw)


def _mpi_env_discovery(port, verbose):
    """Map OpenMPI/MPICH/Slurm env to torch env (reference `comm.py:673-711` uses mpi4py; we read env)."""
    for r, w, lr in (("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),
                     ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"), ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID")):
        if r in os.environ and w in os.environ:
            os.environ["RANK"] = os.environ[r]
            os.environ["WORLD_SIZE"] = os.environ[w]
            os.environ["LOCAL_RANK"] = os.environ.get(lr, "0")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(port))
            if verbose:
                logger.info(f"Discovered MPI-style env via {r}: rank={os.environ['RANK']} world={os.environ['WORLD_SIZE']}")
            return True
    return False


def mpi_discovery(distributed_port=TORCH_DISTRIBUTED_DEFAULT_PORT, verbose=True):
    """Reference name (`comm.py:673`): the launcher env of OpenMPI / MPICH / Slurm mapped to the torch env vars
    (mpi4py is not part of this stack; the MPI launchers export everything needed)."""
    if not _mpi_env_discovery(distributed_port, verbose):
        raise RuntimeError("mpi_discovery: no OpenMPI / MPICH / Slurm rank variables in the environment")
    if is_initialized():
        assert get_rank() == int(os.environ["RANK"]) and get_world_size() == int(os.environ["WORLD_SIZE"]), \
            "MPI rank / world size disagree with the initialised process group"


def in_aml():
    """Azure Machine Learning job (reference `comm.py:714`)."""
    return "AZUREML_EXPERIMENT_ID" in os.environ


def in_aws_sm():
    """AWS SageMaker job."""
    return "SM_TRAINING_ENV" in os.environ


def in_dlts():
    return "DLTS_JOB_ID" in os.environ


def patch_aml_env_for_torch_nccl_backend(master_port=6105, verbose=True):
    """AzureML exports OpenMPI ranks and its own master-node variables (reference `comm.py:729-760`)."""
    os.environ["RANK"] = os.environ["OMPI_COMM_WORLD_RANK"]
    os.environ["WORLD_SIZE"] = os.environ["OMPI_COMM_WORLD_SIZE"]
    os.environ["LOCAL_RANK"] = os.environ["OMPI_COMM_WORLD_LOCAL_RANK"]
    single_node = int(os.environ.get("OMPI_COMM_WORLD_LOCAL_SIZE", os.environ["WORLD_SIZE"])) == \
        int(os.environ["WORLD_SIZE"])
    if single_node:
        os.environ["MASTER_ADDR"] = os.environ.get("AZ_BATCHAI_MPI_MASTER_NODE", "127.0.0.1")
        os.environ["MASTER_PORT"] = os.environ.get("MASTER_PORT", "54965")
    else:
        os.environ["MASTER_ADDR"] = os.environ["AZ_BATCH_MASTER_NODE"].split(":")[0]
        os.environ.setdefault("MASTER_PORT", str(master_port))
    os.environ["NCCL_SOCKET_IFNAME"] = os.environ.get("NCCL_SOCKET_IFNAME", "^docker0,lo")
    if verbose:
        logger.info(f"AzureML env: rank={os.environ['RANK']} local_rank={os.environ['LOCAL_RANK']} "
                    f"world={os.environ['WORLD_SIZE']} master={os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}")


def patch_aws_sm_env_for_torch_nccl_backend(verbose=True):
    """SageMaker exports OpenMPI ranks; MASTER_ADDR / MASTER_PORT come from the job (reference `comm.py:763-771`)."""
    os.environ["RANK"] = os.environ["OMPI_COMM_WORLD_RANK"]
    os.environ["LOCAL_RANK"] = os.environ["OMPI_COMM_WORLD_LOCAL_RANK"]
    os.environ["WORLD_SIZE"] = os.environ["OMPI_COMM_WORLD_SIZE"]
    if verbose:
        logger.info(f"SageMaker env: rank={os.environ['RANK']} world={os.environ['WORLD_SIZE']}")


def set_backend():
    """API parity (reference `comm.py:198`): there is one backend here, torch.distributed over RCCL / gloo."""
    return None


def init_deepspeed_backend(ds_backend=None, timeout=default_pg_timeout, init_method=None):
    """API parity (reference `comm.py:143`, whose only native backend is oneCCL): nothing beyond torch.distributed
    is initialised here; the xGMI inference all-reduce sets itself up lazily (comm/xgmi.py)."""
    return None


def destroy_process_group(group=None):
    if is_initialized():
        tdist.destroy_process_group(group)


# ---------------------------------------------------------------------------------------------- queries
def get_rank(group=None):
    return tdist.get_rank(group) if is_initialized() else 0


def get_world_size(group=None):
    return tdist.get_world_size(group) if is_initialized() else 1


def get_local_rank():
    return int(os.environ.get("LOCAL_RANK", "0"))


def get_global_rank(group=None, group_rank=0):
    if group is None or not is_initialized():
        return group_rank
    return tdist.get_global_rank(group, group_rank)


def get_world_group():
    return tdist.group.WORLD


def get_all_ranks_from_group(group=None):
    return tdist.get_process_group_ranks(group) if group is not None else list(range(get_world_size()))


def new_group(ranks=None, **kw):
    return tdist.new_group(ranks, **kw)


def get_backend(group=None):
    return tdist.get_backend(group)


def has_all_gather_into_tensor():
    return True


def has_reduce_scatter_tensor():
    return True


def has_coalescing_manager():
    return hasattr(tdist, "_coalescing_manager")


# ---------------------------------------------------------------------------------------------- collectives
@timed_op
def broadcast(tensor, src, group=None, async_op=False, **kw):
    return tdist.broadcast(tensor, src, group=group, async_op=async_op)


@timed_op
def all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False, **kw):
    return tdist.all_reduce(tensor, op=op, group=group, async_op=async_op)


@timed_op
def inference_all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False, **kw):
    """Tensor-parallel decode all-reduce (reference `deepspeed/comm/comm.py` inference_all_reduce). SUM over one
    node takes the native paths of `comm/xgmi.py` — peer-mapped xGMI kernel for device tensors (capturable, no host
    sync), POSIX-shm reduce for host tensors — and falls back to RCCL / gloo otherwise."""
    if op == ReduceOp.SUM and not async_op and is_initialized():
        from . import xgmi
        if xgmi.fast_all_reduce(tensor, group):
            return None
    return tdist.all_reduce(tensor, op=op, group=group, async_op=async_op)


def has_all_reduce_coalesced():
    return hasattr(tdist, "all_reduce_coalesced")


def all_gather_coalesced(output_tensors, input_tensors, group=None, async_op=False):
    """Per-tensor all-gathers issued as one coalesced batch (reference `comm.py:250`)."""
    with tdist._coalescing_manager(group=group, async_ops=async_op) as cm:
        for out, inp in zip(output_tensors, input_tensors):
            tdist.all_gather_into_tensor(out, inp, group=group)
    return cm if async_op else None


@timed_op
def all_reduce_coalesced(tensors, op=ReduceOp.SUM, group=None, async_op=False, **kw):
    return tdist.all_reduce_coalesced(tensors, op=op, group=group, async_op=async_op)


@timed_op
def reduce(tensor, dst, op=ReduceOp.SUM, group=None, async_op=False, **kw):
    return tdist.reduce(tensor, dst, op=op, group=group, async_op=async_op)


@timed_op
def all_gather(tensor_list, tensor, group=None, async_op=False, **kw):
    return tdist.all_gather(tensor_list, tensor, group=group, async_op=async_op)


@timed_op
def all_gather_into_tensor(output_tensor, input_tensor, group=None, async_op=False, **kw):
    return tdist.all_gather_into_tensor(output_tensor, input_tensor, group=group, async_op=async_op)


def allgather_fn(output_tensor, input_tensor, group=None, async_op=False, debug=False):
    return all_gather_into_tensor(output_tensor, input_tensor, group=group, async_op=async_op)


@timed_op
def reduce_scatter_tensor(output_tensor, input_tensor, op=ReduceOp.SUM, group=None, async_op=False, **kw):
    return tdist.reduce_scatter_tensor(output_tensor, input_tensor, op=op, group=group, async_op=async_op)


@timed_op
def reduce_scatter(output, input_list, op=ReduceOp.SUM, group=None, async_op=False, **kw):
    return tdist.reduce_scatter(output, input_list, op=op, group=group, async_op=async_op)


def reduce_scatter_fn(output_tensor, tensor, op=ReduceOp.SUM, group=None, async_op=False, debug=False):
    return reduce_scatter_tensor(output_tensor, tensor, op=op, group=group, async_op=async_op)


@timed_op
def all_to_all_single(output, tensor, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False,
                      **kw):
    return tdist.all_to_all_single(output, tensor, output_split_sizes=output_split_sizes,
                                   input_split_sizes=input_split_sizes, group=group, async_op=async_op)


@timed_op
def all_to_all(output_tensor_list, input_tensor_list, group=None, async_op=False, **kw):
    return tdist.all_to_all(output_tensor_list, input_tensor_list, group=group, async_op=async_op)


@timed_op
def send(tensor, dst, group=None, tag=0, **kw):
    return tdist.send(tensor, dst, group=group, tag=tag)


@timed_op
def recv(tensor, src=None, group=None, tag=0, **kw):
    return tdist.recv(tensor, src, group=group, tag=tag)


@timed_op
def isend(tensor, dst, group=None, tag=0, **kw):
    return tdist.isend(tensor, dst, group=group, tag=tag)


@timed_op
def irecv(tensor, src=None, group=None, tag=0, **kw):
    return tdist.irecv(tensor, src, group=group, tag=tag)


def batch_isend_irecv(p2p_op_list):
    return tdist.batch_isend_irecv(p2p_op_list)


P2POp = tdist.P2POp


@timed_op
def gather(tensor, gather_list=None, dst=0, group=None, async_op=False, **kw):
    return tdist.gather(tensor, gather_list, dst, group=group, async_op=async_op)


@timed_op
def scatter(tensor, scatter_list=None, src=0, group=None, async_op=False, **kw):
    return tdist.scatter(tensor, scatter_list, src, group=group, async_op=async_op)


def barrier(group=None, async_op=False, device_ids=None):
    if not is_initialized():
        return None
    if get_backend(group) == "nccl" and device_ids is None:
        device_ids = [torch.cuda.current_device()]
    return tdist.barrier(group=group, async_op=async_op, device_ids=device_ids)


def monitored_barrier(group=None, timeout=None, wait_all_ranks=False):
    return tdist.monitored_barrier(group=group, timeout=timeout, wait_all_ranks=wait_all_ranks)


def all_gather_object(object_list, obj, group=None):
    return tdist.all_gather_object(object_list, obj, group=group)


def broadcast_object_list(object_list, src=0, group=None, device=None):
    return tdist.broadcast_object_list(object_list, src=src, group=group, device=device)


def log_summary(show_straggler=False):
    barrier()
    if get_rank() == 0:
        comms_logger.log_all(print_log=True, show_straggler=show_straggler)
    barrier()


# ------------------------------------------------------------------------------------------------ backend object
def get_local_rank_from_launcher():
    return int(os.environ.get("LOCAL_RANK", os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", 0)))


def get_world_rank_from_launcher():
    return int(os.environ.get("RANK", os.environ.get("OMPI_COMM_WORLD_RANK", 0)))


def get_world_size_from_launcher():
    return int(os.environ.get("WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_SIZE", 1)))


class TorchBackend:
    """torch.distributed as a backend object (reference `comm/torch.py:99`): every collective of this module as a
    method, for code that holds a backend instead of calling the module functions."""

    def __init__(self, backend=None, timeout=default_pg_timeout, init_method=None, rank=-1, world_size=-1,
                 name="torch"):
        self.name = name
        self.single_gpu_mode = True
        if not is_initialized():
            init_distributed(dist_backend=backend, timeout=timeout, init_method=init_method, rank=rank,
                             world_size=world_size)
        self.using_mpi = False
        self.initialized = True

    def is_initialized(self):
        return is_initialized()

    def has_all_gather_into_tensor(self):
        return hasattr(tdist, "all_gather_into_tensor")

    def has_reduce_scatter_tensor(self):
        return hasattr(tdist, "reduce_scatter_tensor")

    def has_all_reduce_coalesced(self):
        return has_all_reduce_coalesced()

    def __getattr__(self, name):
        # every collective / query of this module (all_reduce, all_gather_into_tensor, get_rank, new_group, ...)
        fn = globals().get(name)
        if callable(fn) and not name.startswith("_"):
            return fn
        raise AttributeError(name)

