"""`zero.Init` (construct a model already partitioned) and `GatheredParameters` (temporarily materialise partitioned
params), reference `runtime/zero/partition_parameters.py:303-2134`.

Init: while active, tensors are created on the accelerator (the default device is switched, the reference patches
the tensor constructors for the same effect, `:373-555`), and every nn.Module's `__init__` is post-processed: its
freshly created parameters are cast to the training dtype, made identical across ranks (broadcast from rank 0, as
the reference does at `:423`) and reduced to this rank's 1/dp slice `p.ds_tensor`; `p.data` becomes empty. At most
one module's parameters exist in full at any time (never on the host), so a 70B model can be built on a node whose
per-GPU memory only holds its shard. `DeepSpeedEngine` then regroups these per-parameter shards into its flat
groups one parameter at a time.

Per-parameter API (reference `:1336-1338` `all_gather` / `partition` + `ds_*` attributes): every partitioned param
carries `ds_shape`, `ds_numel`, `ds_status` and the methods `p.all_gather(param_list=None)` / `p.partition(
param_list=None)` (materialise / drop outside a `GatheredParameters` block).

`register_external_parameter(module, param)`: `module`'s forward uses a parameter owned by another module (tied
embeddings, shared projections). Under ZeRO-3 the fetch hooks of `module` then gather that parameter's group too
(reference `partition_parameters.py` register_external_parameter + `parameter_offload.py` external params).
"""
import functools

from enum import Enum

import torch
import torch.nn as nn

from ... import comm as dist
from ...accelerator import get_accelerator
from ...parallel import groups
from .flat_optimizer import ZeroParamStatus

_init_depth = 0


def _ceil(a, b):
    return (a + b - 1) // b


_active_inits = []


def shutdown_init_context():
    """Suspend an active `zero.Init` (reference `partition_parameters.py:shutdown_init_context`, called by
    `initialize()` so modules the engine builds internally are not partitioned)."""
    for ctx in _active_inits:
        ctx._suspend()


def restore_init_context():
    for ctx in _active_inits:
        ctx._resume()


# ------------------------------------------------------------------------------------------------ per-param API
def _param_all_gather(p, param_list=None, async_op=False):
    params = [p] if param_list is None else list(param_list)
    ctx = GatheredParameters(params)
    ctx.__enter__()
    for q in ctx.params:
        q.__dict__["_ds_gather_ctx"] = ctx
    return None


def _param_partition(p, param_list=None, has_been_updated=False):
    params = [p] if param_list is None else list(param_list)
    done = set()
    for q in params:
        ctx = q.__dict__.pop("_ds_gather_ctx", None)
        if ctx is not None and id(ctx) not in done:
            done.add(id(ctx))
            ctx.__exit__(None, None, None)


def _attach_api(p):
    p.all_gather = functools.partial(_param_all_gather, p)
    p.partition = functools.partial(_param_partition, p)


# ------------------------------------------------------------------------------------------------ external params
def register_external_parameter(module, parameter):
    """Declare that `module`'s forward uses `parameter` although another module owns it."""
    if not isinstance(parameter, nn.Parameter):
        raise RuntimeError("register_external_parameter: parameter must be a torch.nn.Parameter")
    ext = module.__dict__.setdefault("_ds_external_params", [])
    if all(q is not parameter for q in ext):
        ext.append(parameter)
    g = getattr(parameter, "ds_group", None)
    coord = getattr(getattr(g, "_opt", None), "coordinator", None) if g is not None else None
    if coord is not None:
        coord.install_external(module)


def unregister_external_parameter(module, parameter):
    ext = module.__dict__.get("_ds_external_params", [])
    module.__dict__["_ds_external_params"] = [q for q in ext if q is not parameter]


class ZeroParamType(Enum):
    NORMAL = 1     # partitioned across the data-parallel group
    PARTITIONED = 2
    REMOTE = 3     # lives on another device (host / NVMe) until fetched


class AllGatherHandle:
    """Completion handle of one parameter gather (reference `partition_parameters.py:620-640`). Gathers here are
    issued per flat group on the all-gather stream; the handle carries the event compute must wait for."""

    def __init__(self, handle, param, quantization=None):
        self.handle, self.param, self.quantization = handle, param, quantization

    def wait(self):
        if self.handle is not None and hasattr(self.handle, "wait"):
            self.handle.wait()
        if hasattr(self.param, "ds_status"):
            self.param.ds_status = ZeroParamStatus.AVAILABLE


class AllGatherCoalescedHandle:

    def __init__(self, allgather_handle, params, partitions=None, world_size=1, use_secondary_tensor=False,
                 forward=False, quantization=None):
        self.allgather_handle, self.params = allgather_handle, list(params)
        self.complete = False

    def wait(self):
        if self.complete:
            return
        if self.allgather_handle is not None and hasattr(self.allgather_handle, "wait"):
            self.allgather_handle.wait()
        for p in self.params:
            if hasattr(p, "ds_status"):
                p.ds_status = ZeroParamStatus.AVAILABLE
        self.complete = True


class NoGatherHandle(AllGatherHandle):
    """Handle for a single-rank group: nothing to wait for."""

    def __init__(self, param):
        super().__init__(None, param)


class NoGatherCoalescedHandle(AllGatherCoalescedHandle):

    def __init__(self, params):
        super().__init__(None, params)


class MultipleAllGatherHandles:

    def __init__(self, handles):
        self.handles = list(handles)

    def wait(self):
        for h in self.handles:
            h.wait()


def free_param(param):
    """Drop the gathered data of a ZeRO-3 parameter (its partition stays)."""
    if hasattr(param, "partition"):
        param.partition()
    else:
        param.data = torch.empty(0, dtype=param.dtype, device=param.device)


def print_rank_0(message, debug=False, force=False):
    if (debug or force) and (not dist.is_initialized() or dist.get_rank() == 0):
        print(message)


def is_zero_param(p):
    return hasattr(p, "ds_tensor") or hasattr(p, "ds_group")


@torch.no_grad()
def _partition_param(p, dp, rank, group, device, dtype):
    if hasattr(p, "ds_tensor"):
        return
    data = p.data.to(device=device, dtype=dtype if p.is_floating_point() else p.dtype)
    if dp > 1:
        dist.broadcast(data, groups._get_broadcast_src_rank() if groups.mpu else 0, group=group)
    n = data.numel()
    per = _ceil(n, dp)
    flat = torch.zeros(per * dp, dtype=data.dtype, device=device)
    flat[:n].copy_(data.reshape(-1))
    p.ds_tensor = flat[rank * per:(rank + 1) * per].clone()
    p.ds_shape = data.shape
    p.ds_numel = n
    p.ds_status = ZeroParamStatus.NOT_AVAILABLE
    p.ds_process_group = group
    p.data = torch.empty(0, dtype=data.dtype, device=device)
    _attach_api(p)


@torch.no_grad()
def gather_partitioned_param(p):
    """Full tensor of a `zero.Init`-partitioned param (not yet adopted by an engine)."""
    group = getattr(p, "ds_process_group", None)
    dp = dist.get_world_size(group)
    full = torch.empty(p.ds_tensor.numel() * dp, dtype=p.ds_tensor.dtype, device=p.ds_tensor.device)
    if dp > 1:
        dist.all_gather_into_tensor(full, p.ds_tensor, group=group)
    else:
        full.copy_(p.ds_tensor)
    return full[:p.ds_numel].view(p.ds_shape)


class Init:
    """Context manager: modules built inside are partitioned at construction (see module docstring)."""

    def __init__(self, module=None, data_parallel_group=None, mem_efficient_linear=True, remote_device=None,
                 pin_memory=False, config_dict_or_path=None, config=None, enabled=True, dtype=None, mpu=None,
                 zero_param_parallel_group=None, zero_quantized_weights=False, zero_quantized_nontrainable_weights=False,
                 sequence_data_parallel_group=None, param_swapper=None):
        self.enabled = enabled
        if not enabled:
            return
        if not dist.is_initialized():
            dist.init_distributed()
        self.group = sequence_data_parallel_group or data_parallel_group or groups._get_sequence_data_parallel_group()
        self.dp = dist.get_world_size(self.group)
        self.rank = dist.get_rank(self.group)
        acc = get_accelerator()
        self.device = torch.device("cuda", acc.current_device()) if acc.device_name() == "cuda" else \
            torch.device("cpu")
        if remote_device == "cpu":
            self.device = torch.device("cpu")
        if dtype is None:
            cfg = config_dict_or_path or config
            dtype = torch.float32
            if isinstance(cfg, dict):
                if cfg.get("bf16", {}).get("enabled"):
                    dtype = torch.bfloat16
                elif cfg.get("fp16", {}).get("enabled"):
                    dtype = torch.float16
        self.dtype = dtype
        if module is not None:
            self._convert(module)

    def get_dp_process_group(self):
        """The group parameters are partitioned over (reference `partition_parameters.py:968`)."""
        return self.group

    def get_partition_dp_group(self, param=None):
        return getattr(param, "ds_process_group", self.group) if param is not None else self.group

    def get_partition_rank(self):
        return self.rank

    @property
    def num_partitions(self):
        return self.dp

    def _convert(self, module):
        for m in module.modules():
            for p in m.parameters(recurse=False):
                _partition_param(p, self.dp, self.rank, self.group, self.device, self.dtype)

    def _suspend(self):
        self._suspended = True
        if getattr(self, "_prev_device", None) is not None:
            torch.set_default_device(self._prev_device)

    def _resume(self):
        self._suspended = False
        if getattr(self, "_prev_device", None) is not None:
            torch.set_default_device(self.device)

    def __enter__(self):
        global _init_depth
        if not self.enabled:
            return self
        _init_depth += 1
        self._suspended = False
        _active_inits.append(self)
        # born on the accelerator: module constructors allocate straight into device memory
        self._prev_device = None
        if self.device.type != "cpu":
            self._prev_device = torch.get_default_device()
            torch.set_default_device(self.device)
        self._orig_init = nn.Module.__init__
        ctx = self
        orig = self._orig_init

        # patch every Module subclass' __init__ through the base: convert params owned directly by the module
        self._patched = {}

        def _wrap(cls):
            init = cls.__dict__.get("__init__")
            if init is None or getattr(init, "_ds_wrapped", False):
                return

            @functools.wraps(init)
            def wrapped(module, *a, **k):
                init(module, *a, **k)
                if ctx._suspended:
                    return
                for p in module.parameters(recurse=False):
                    _partition_param(p, ctx.dp, ctx.rank, ctx.group, ctx.device, ctx.dtype)

            wrapped._ds_wrapped = True
            self._patched[cls] = init
            cls.__init__ = wrapped

        def _all_subclasses(c):
            out = set()
            for s in c.__subclasses__():
                out.add(s)
                out |= _all_subclasses(s)
            return out

        for cls in _all_subclasses(nn.Module):
            _wrap(cls)
        self._wrap = _wrap
        # classes defined inside the context get wrapped on subclass creation
        self._had_init_subclass = "__init_subclass__" in nn.Module.__dict__
        self._orig_init_subclass = nn.Module.__dict__.get("__init_subclass__")

        def init_subclass(cls, **kw):
            _wrap(cls)

        nn.Module.__init_subclass__ = classmethod(init_subclass)
        return self

    def __exit__(self, *exc):
        global _init_depth
        if not self.enabled:
            return False
        for cls, init in self._patched.items():
            cls.__init__ = init
        if self._prev_device is not None:
            torch.set_default_device(self._prev_device)
        if self in _active_inits:
            _active_inits.remove(self)
        if self._had_init_subclass:
            nn.Module.__init_subclass__ = self._orig_init_subclass
        else:
            del nn.Module.__init_subclass__
        _init_depth -= 1
        return False


class GatheredParameters:
    """Materialise partitioned params inside the block; with `modifier_rank`, changes made on that rank are
    broadcast and written back into every rank's shard and fp32 master on exit."""

    def __init__(self, params, modifier_rank=None, fwd_module=None, enabled=True):
        if isinstance(params, nn.Parameter) or torch.is_tensor(params):
            params = [params]
        self.params = [p for p in params if is_zero_param(p)]
        self.modifier_rank = modifier_rank
        self.enabled = enabled and len(self.params) > 0
        self._gathered_groups = []
        self._gathered_init = []

    def __enter__(self):
        if not self.enabled:
            return self
        seen = set()
        for p in self.params:
            g = getattr(p, "ds_group", None)
            if g is not None:
                if id(g) in seen:
                    continue
                seen.add(id(g))
                if g.status != ZeroParamStatus.AVAILABLE:
                    opt = g._opt
                    full = torch.empty(g.padded, dtype=g.dtype, device=g.device)
                    shard = g.shard if g.shard.device == full.device else g.shard.to(full.device)  # offload_param
                    if g.partition:
                        dist.all_gather_into_tensor(full, shard, group=g.dp_group)
                    else:
                        full.copy_(shard)
                    g.full = full
                    opt._point_params(g)
                    g.status = ZeroParamStatus.AVAILABLE
                    self._gathered_groups.append(g)
            elif hasattr(p, "ds_tensor") and p.data.numel() != p.ds_numel:
                p.data = gather_partitioned_param(p).clone()
                self._gathered_init.append(p)
        return self

    def __exit__(self, *exc):
        if not self.enabled:
            return False
        if self.modifier_rank is not None:
            for p in self.params:
                g = getattr(p, "ds_group", None)
                grp = g.dp_group if g is not None else getattr(p, "ds_process_group", None)
                if dist.get_world_size(grp) > 1:
                    dist.broadcast(p.data, dist.get_global_rank(grp, self.modifier_rank), group=grp)
                if g is not None:
                    g._opt.set_full_fp32_param(p, p.data)
                elif hasattr(p, "ds_tensor"):
                    dp = dist.get_world_size(getattr(p, "ds_process_group", None))
                    r = dist.get_rank(getattr(p, "ds_process_group", None))
                    per = p.ds_tensor.numel()
                    flat = torch.zeros(per * dp, dtype=p.ds_tensor.dtype, device=p.ds_tensor.device)
                    flat[:p.ds_numel].copy_(p.data.reshape(-1))
                    p.ds_tensor.copy_(flat[r * per:(r + 1) * per])
        for g in self._gathered_groups:
            g._opt._release_params(g)
            g.full = None
        for p in self._gathered_init:
            p.data = torch.empty(0, dtype=p.ds_tensor.dtype, device=p.ds_tensor.device)
        return False
