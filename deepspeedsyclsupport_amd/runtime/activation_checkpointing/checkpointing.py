"""Activation checkpointing with partitioned / host-offloaded checkpoints (reference
`runtime/activation_checkpointing/checkpointing.py:122-1162`).

API parity: `checkpoint(function, *args)`, `non_reentrant_checkpoint`, `configure(...)`, `is_configured`, `reset`,
`set_num_layers`, `get_cuda_rng_tracker`, `model_parallel_cuda_manual_seed`, `CheckpointFunction`.

MI355X notes:
* `partition_activations`: each saved layer input is split across the tensor-parallel group (1/mp per rank) and
  re-assembled with one `all_gather_into_tensor` over xGMI right before recompute.
* `cpu_checkpointing`: saved inputs go to pinned host memory with a non-blocking D2H on a side HIP stream (overlaps the
  next layer's forward); the backward issues the H2D prefetch on the same stream and the compute stream waits on an
  event only when the tensor is needed. With 288 GB of HBM this is rarely required below 70B.
* `contiguous_memory_optimization` (reference `:373-483`): the partitioned checkpoints of one iteration live in
  pre-allocated `[number_checkpoints, partition]` buffers, one per (argument position, size, dtype, residence), filled
  slot by slot as layers checkpoint and rewound by `reset()` at the iteration boundary — no allocator traffic and no
  fragmentation from thousands of odd-sized slices. Host-resident buffers are pinned once.
* `non_reentrant_checkpoint` (reference `:724`): saved-tensor hooks discard the segment's activations in forward and
  recompute them on first use in backward; the segment INPUTS are kept by the same `_Saved` records as the reentrant
  path, so `partition_activations`, `cpu_checkpointing` and the contiguous buffers apply to both variants.
* RNG: the HIP generator state is captured per checkpoint and restored around recompute, so dropout masks match.
"""
import contextlib

import torch

from ... import comm as dist
from ...accelerator import get_accelerator
from ...utils.logging import logger

deepspeed_checkpointing_enabled = False
mpu = None
mp_rank = 0
mp_size = 1
mp_group = None
num_layers = None
PARTITION_ACTIVATIONS = False
CPU_CHECKPOINT = False
CONTIGUOUS_CHECKPOINTING = False
SYNCHRONIZE = False
PROFILE_TIME = False
_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"
_side_stream = None


def _device_rng_state():
    acc = get_accelerator()
    return acc.get_rng_state() if acc.device_name() == "cuda" else None


def _set_device_rng_state(state):
    if state is not None:
        get_accelerator().set_rng_state(state)


class CudaRNGStatesTracker:
    """Named RNG states so tensor-parallel regions use different dropout streams (reference `:122-191`)."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = states

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception(f"seed {seed} already exists")
        self.seeds_.add(seed)
        if name in self.states_:
            raise Exception(f"cuda rng state {name} already exists")
        orig = _device_rng_state()
        get_accelerator().manual_seed(seed)
        self.states_[name] = _device_rng_state()
        _set_device_rng_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception(f"cuda rng state {name} is not added")
        orig = _device_rng_state()
        _set_device_rng_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _device_rng_state()
            _set_device_rng_state(orig)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


def model_parallel_cuda_manual_seed(seed):
    global mpu
    tp_rank = mpu.get_model_parallel_rank() if mpu is not None else 0
    offset = seed + 2718
    model_parallel_seed = offset + tp_rank
    data_parallel_seed = seed
    _CUDA_RNG_STATE_TRACKER.reset()
    get_accelerator().manual_seed(data_parallel_seed)
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, model_parallel_seed)


def model_parallel_reconfigure_tp_seed(seed):
    global mpu
    tp_rank = mpu.get_model_parallel_rank() if mpu is not None else 0
    with _CUDA_RNG_STATE_TRACKER.fork():
        get_accelerator().manual_seed(seed + 2718 + tp_rank)


def detach_variable(inputs, device=None):
    out = []
    for x in inputs:
        if torch.is_tensor(x):
            y = x.detach() if device is None else x.detach().to(device)
            y.requires_grad = x.requires_grad
            out.append(y)
        else:
            out.append(x)
    return tuple(out)


# ---------------------------------------------------------------------------------------------- saving inputs
def _side():
    global _side_stream
    if _side_stream is None and get_accelerator().device_name() == "cuda":
        _side_stream = get_accelerator().Stream()
    return _side_stream


class _ContiguousPool:
    """Pre-allocated checkpoint storage: one `[slots, numel]` buffer per (argument position, numel, dtype, device /
    pinned host), a cursor per buffer that `rewind()` resets every iteration. A buffer grows (doubling) when an
    iteration checkpoints more segments than `number_checkpoints` announced."""

    def __init__(self):
        self.buffers = {}
        self.cursor = {}
        self.allocations = 0

    def slot(self, arg_idx, numel, dtype, device, pinned):
        key = (arg_idx, int(numel), dtype, str(device), bool(pinned))
        i = self.cursor.get(key, 0)
        buf = self.buffers.get(key)
        if buf is None or i >= buf.shape[0]:
            want = max(int(num_layers or 1), 1) if buf is None else 2 * buf.shape[0]
            new = torch.empty((want, int(numel)), dtype=dtype, device="cpu" if pinned else device,
                              pin_memory=bool(pinned) and get_accelerator().device_name() == "cuda")
            if buf is not None:  # slots already handed out this iteration stay valid in the old buffer
                self.cursor[key] = i = 0
            self.buffers[key] = buf = new
            self.allocations += 1
        self.cursor[key] = i + 1
        return buf[i]

    def rewind(self):
        self.cursor = {}


_POOL = _ContiguousPool()


class _Saved:
    """A checkpoint input stored partitioned across MP and/or in host memory (optionally in the contiguous pool)."""

    def __init__(self, t, arg_idx=0):
        self.requires_grad = t.requires_grad
        self.shape, self.dtype, self.device = t.shape, t.dtype, t.device
        data = t.detach()
        self.partitioned = PARTITION_ACTIVATIONS and mp_size > 1 and data.numel() % mp_size == 0
        self.on_host = CPU_CHECKPOINT and data.is_cuda
        pooled = CONTIGUOUS_CHECKPOINTING and self.partitioned
        self.pooled = pooled
        if self.partitioned:
            flat = data.reshape(-1)
            n = flat.numel() // mp_size
            part = flat[mp_rank * n:(mp_rank + 1) * n]
            if pooled and not self.on_host:
                dst = _POOL.slot(arg_idx, n, data.dtype, data.device, False)
                dst.copy_(part)
                data = dst
            else:
                data = part.clone() if not self.on_host else part
        self.event = None
        if self.on_host:
            s = _side()
            if pooled:
                host = _POOL.slot(arg_idx, data.numel(), data.dtype, data.device, True).view(data.shape)
            else:
                host = torch.empty(data.shape, dtype=data.dtype, pin_memory=True)
            s.wait_stream(get_accelerator().current_stream())
            with get_accelerator().stream(s):
                host.copy_(data, non_blocking=True)
                data.record_stream(s)
            self.event = get_accelerator().Event()
            self.event.record(s)
            data = host
        self.data = data

    def restore(self):
        data = self.data
        if self.on_host:
            s = _side()
            self.event.synchronize()
            with get_accelerator().stream(s):
                dev = data.to(self.device, non_blocking=True)
            get_accelerator().current_stream().wait_stream(s)
            dev.record_stream(get_accelerator().current_stream())
            data = dev
        if self.partitioned:
            full = torch.empty(data.numel() * mp_size, dtype=data.dtype, device=data.device)
            dist.all_gather_into_tensor(full, data.contiguous(), group=mp_group)
            data = full
        out = data.reshape(self.shape).detach()
        out.requires_grad = self.requires_grad
        return out


class CheckpointFunction(torch.autograd.Function):
    """Reentrant checkpoint: forward without graph, recompute in backward."""

    @staticmethod
    def forward(ctx, run_function, all_outputs, *args):
        ctx.run_function = run_function
        ctx.fwd_cpu_state = torch.get_rng_state()
        ctx.fwd_dev_state = _device_rng_state()
        ctx.fwd_tracker_states = get_cuda_rng_tracker().get_states()
        ctx.saved = [(_Saved(a, i) if torch.is_tensor(a) else a) for i, a in enumerate(args)]
        with torch.no_grad():
            outputs = run_function(*args)
        if SYNCHRONIZE:
            get_accelerator().synchronize()
        if torch.is_tensor(outputs):
            return outputs
        ctx.mark_non_differentiable(*[o for o in outputs if torch.is_tensor(o) and not o.is_floating_point()])
        return tuple(outputs)

    @staticmethod
    def backward(ctx, *grads):
        inputs = [s.restore() if isinstance(s, _Saved) else s for s in ctx.saved]
        bwd_cpu_state = torch.get_rng_state()
        bwd_dev_state = _device_rng_state()
        bwd_tracker_states = get_cuda_rng_tracker().get_states()
        torch.set_rng_state(ctx.fwd_cpu_state)
        _set_device_rng_state(ctx.fwd_dev_state)
        get_cuda_rng_tracker().set_states(ctx.fwd_tracker_states)
        detached = detach_variable(tuple(inputs))
        with torch.enable_grad():
            outputs = ctx.run_function(*detached)
        torch.set_rng_state(bwd_cpu_state)
        _set_device_rng_state(bwd_dev_state)
        get_cuda_rng_tracker().set_states(bwd_tracker_states)
        if torch.is_tensor(outputs):
            outputs = (outputs, )
        outs, gs = [], []
        for o, g in zip(outputs, grads):
            if torch.is_tensor(o) and o.requires_grad and g is not None:
                outs.append(o)
                gs.append(g)
        if outs:
            torch.autograd.backward(outs, gs)
        return (None, None) + tuple(x.grad if torch.is_tensor(x) else None for x in detached)


def checkpoint(function, *args):
    """Checkpoint a model segment (reference `checkpointing.py:989`)."""
    return CheckpointFunction.apply(function, [], *args)


def non_reentrant_checkpoint(function, *args):
    """Non-reentrant checkpoint (reference `:724`): the forward runs WITH a graph whose saved activations are
    discarded by saved-tensor hooks; the first backward node that needs one triggers a recompute of the segment
    (torch's hook machinery, which also stops the recompute as soon as every needed tensor is back). The segment's
    inputs are held the same way as in the reentrant path — partitioned across the tensor-parallel group, in pinned
    host memory, in the contiguous pool — and re-assembled for the recompute; RNG states are replayed so dropout
    repeats."""
    import torch.utils.checkpoint as cp
    holder = {"args": args, "saved": None}
    fwd_cpu_state = torch.get_rng_state()
    fwd_dev_state = _device_rng_state()
    fwd_tracker_states = get_cuda_rng_tracker().get_states()

    def run():
        if holder["args"] is not None:  # the forward pass itself
            return function(*holder["args"])
        inputs = [s.restore() if isinstance(s, _Saved) else s for s in holder["saved"]]
        bwd_cpu_state = torch.get_rng_state()
        bwd_dev_state = _device_rng_state()
        bwd_tracker_states = get_cuda_rng_tracker().get_states()
        torch.set_rng_state(fwd_cpu_state)
        _set_device_rng_state(fwd_dev_state)
        get_cuda_rng_tracker().set_states(fwd_tracker_states)
        try:
            return function(*inputs)
        finally:  # also on the early stop torch raises once the last needed activation is recomputed
            torch.set_rng_state(bwd_cpu_state)
            _set_device_rng_state(bwd_dev_state)
            get_cuda_rng_tracker().set_states(bwd_tracker_states)

    out = cp.checkpoint(run, use_reentrant=False, preserve_rng_state=False)
    holder["saved"] = [(_Saved(a, i) if torch.is_tensor(a) else a) for i, a in enumerate(args)]
    holder["args"] = None
    if SYNCHRONIZE:
        get_accelerator().synchronize()
    return out


def partition_activations_in_checkpoint(partition_activation):
    global PARTITION_ACTIVATIONS
    PARTITION_ACTIVATIONS = partition_activation


def set_num_layers(nlayers):
    global num_layers
    num_layers = nlayers


def reset():
    """Iteration boundary (reference `:1004`): rewind the contiguous checkpoint buffers so the next forward refills
    them from slot 0. Call it once per training step when `contiguous_memory_optimization` is on (the engine does)."""
    _POOL.rewind()


def configure(mpu_, deepspeed_config=None, partition_activations=None, contiguous_checkpointing=None,
              num_checkpoints=None, checkpoint_in_cpu=None, synchronize=None, profile=None):
    global mpu, mp_rank, mp_size, mp_group, PARTITION_ACTIVATIONS, CONTIGUOUS_CHECKPOINTING, CPU_CHECKPOINT
    global SYNCHRONIZE, PROFILE_TIME, num_layers, deepspeed_checkpointing_enabled
    deepspeed_checkpointing_enabled = True
    if deepspeed_config is not None:
        from ..config import DeepSpeedConfig
        cfg = deepspeed_config if isinstance(deepspeed_config, DeepSpeedConfig) else DeepSpeedConfig(deepspeed_config)
        ac = cfg.activation_checkpointing_config
        PARTITION_ACTIVATIONS = ac.partition_activations
        CONTIGUOUS_CHECKPOINTING = ac.contiguous_memory_optimization
        num_layers = ac.number_checkpoints
        CPU_CHECKPOINT = ac.cpu_checkpointing
        SYNCHRONIZE = ac.synchronize_checkpoint_boundary
        PROFILE_TIME = ac.profile
    if partition_activations is not None:
        PARTITION_ACTIVATIONS = partition_activations
    if contiguous_checkpointing is not None:
        CONTIGUOUS_CHECKPOINTING = contiguous_checkpointing
    if num_checkpoints is not None:
        num_layers = num_checkpoints
    if checkpoint_in_cpu is not None:
        CPU_CHECKPOINT = checkpoint_in_cpu
    if synchronize is not None:
        SYNCHRONIZE = synchronize
    if profile is not None:
        PROFILE_TIME = profile
    mpu = mpu_
    if mpu is not None:
        mp_rank = mpu.get_model_parallel_rank()
        mp_size = mpu.get_model_parallel_world_size()
        mp_group = mpu.get_model_parallel_group()
    else:
        mp_rank, mp_size, mp_group = 0, 1, None
    if CONTIGUOUS_CHECKPOINTING:
        assert PARTITION_ACTIVATIONS, "Contiguous Checkpointing is only available with partitioned activations."
        assert num_layers is not None, "Must specify the number of layers with contiguous memory checkpointing"


def is_configured():
    return deepspeed_checkpointing_enabled
