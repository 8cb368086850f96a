"""Device facade: exactly one GPU path (ROCm/HIP via torch.cuda) plus a CPU path for plumbing tests.

The reference multiplexes seven accelerators behind an ABC with ~55 methods and runtime auto-detection
(`accelerator/abstract_accelerator.py:10-277`, `accelerator/real_accelerator.py:51-192`). On MI355X there is
nothing to multiplex: if a HIP device is visible we run on it with RCCL (`"nccl"` backend name on ROCm);
otherwise (CI containers, `gloo` plumbing tests) we run on the host. `DS_ACCELERATOR=cpu` forces the host path.

Only methods the framework actually uses are provided, with the reference's names so user code that calls
`get_accelerator().device_name()` etc. keeps working.
"""
import functools
import os

import torch


class _Base:
    _name = "base"
    _comm = "gloo"

    # ------------------------------------------------------------------ identity
    def device_name(self, device_index=None):
        if device_index is None:
            return self._name
        return f"{self._name}:{device_index}"

    def communication_backend_name(self):
        return self._comm

    def is_synchronized_device(self):
        return self._name == "cpu"

    def use_host_timers(self):
        return self.is_synchronized_device()

    def resolves_data_dependency(self):
        return self.is_synchronized_device()

    def handles_memory_backpressure(self):
        return self.is_synchronized_device()

    def device(self, device_index=None):
        return torch.device(self.device_name(device_index))

    def current_device_name(self):
        return self.device_name(self.current_device())

    # ------------------------------------------------------------------ dtypes
    def is_bf16_supported(self):
        return True

    def is_fp16_supported(self):
        return True

    def supported_dtypes(self):
        return [torch.float32, torch.bfloat16, torch.float16]

    # ------------------------------------------------------------------ misc
    def range_push(self, msg):
        pass

    def range_pop(self):
        pass

    def lazy_call(self, callback):
        return callback()

    def on_accelerator(self, tensor):
        return tensor.device.type == self._name.split(":")[0]

    def op_builder_dir(self):
        return "deepspeedsyclsupport_amd.ops"

    # ------------------------------------------------------------------ op builders (reference
    # `accelerator/abstract_accelerator.py:249-266`): one in-tree builder table serves every name
    def get_op_builder(self, class_name):
        from .ops import op_builder
        return getattr(op_builder, class_name, None)

    def create_op_builder(self, class_name):
        cls = self.get_op_builder(class_name)
        return None if cls is None else cls()

    def build_extension(self):
        from torch.utils.cpp_extension import BuildExtension
        return BuildExtension

    def export_envs(self):
        """Environment variable prefixes the launcher forwards to remote ranks."""
        return ["NCCL", "RCCL", "HSA", "HIP", "ROCR", "GPU_", "PYTORCH_"]

    def is_triton_supported(self):
        return False  # no Triton path in this framework: every kernel is in-tree HIP

    def random(self):
        return torch.random

    def amp(self):
        return getattr(torch, "amp", None)

    # ------------------------------------------------------------------ legacy tensor constructors
    def _tensor_type(self, dtype):
        import functools
        return functools.partial(torch.tensor, dtype=dtype, device=self.current_device_name())

    @property
    def BFloat16Tensor(self):
        return self._tensor_type(torch.bfloat16)

    @property
    def ByteTensor(self):
        return self._tensor_type(torch.uint8)

    @property
    def DoubleTensor(self):
        return self._tensor_type(torch.float64)

    @property
    def FloatTensor(self):
        return self._tensor_type(torch.float32)

    @property
    def HalfTensor(self):
        return self._tensor_type(torch.float16)

    @property
    def IntTensor(self):
        return self._tensor_type(torch.int32)

    @property
    def LongTensor(self):
        return self._tensor_type(torch.int64)

    # ------------------------------------------------------------------ older memory-stat names
    def memory_cached(self, device_index=None):
        return self.memory_reserved(device_index)

    def max_memory_cached(self, device_index=None):
        return self.max_memory_reserved(device_index)

    def reset_max_memory_cached(self, device_index=None):
        return self.reset_peak_memory_stats(device_index)


class RocmAccelerator(_Base):
    """MI355X (gfx950) through PyTorch-ROCm: `torch.cuda` is the HIP runtime, `nccl` is RCCL."""
    _name = "cuda"
    _comm = "nccl"

    def is_available(self):
        return torch.cuda.is_available()

    def device_count(self):
        return torch.cuda.device_count()

    def current_device(self):
        return torch.cuda.current_device()

    def set_device(self, device_index):
        torch.cuda.set_device(device_index)

    def synchronize(self, device_index=None):
        torch.cuda.synchronize(device_index)

    # RNG
    def manual_seed(self, seed):
        torch.cuda.manual_seed(seed)

    def manual_seed_all(self, seed):
        torch.cuda.manual_seed_all(seed)

    def get_rng_state(self, device_index=None):
        return torch.cuda.get_rng_state(device_index or "cuda")

    def set_rng_state(self, new_state, device_index=None):
        return torch.cuda.set_rng_state(new_state, device_index or "cuda")

    def initial_seed(self):
        return torch.cuda.initial_seed()

    def default_generator(self, device_index):
        return torch.cuda.default_generators[device_index]

    # streams / events
    @property
    def Stream(self):
        return torch.cuda.Stream

    def stream(self, stream):
        return torch.cuda.stream(stream)

    def current_stream(self, device_index=None):
        return torch.cuda.current_stream(device_index)

    def default_stream(self, device_index=None):
        return torch.cuda.default_stream(device_index)

    @property
    def Event(self):
        return torch.cuda.Event

    # memory
    def empty_cache(self):
        torch.cuda.empty_cache()

    def memory_allocated(self, device_index=None):
        return torch.cuda.memory_allocated(device_index)

    def max_memory_allocated(self, device_index=None):
        return torch.cuda.max_memory_allocated(device_index)

    def reset_max_memory_allocated(self, device_index=None):
        return torch.cuda.reset_peak_memory_stats(device_index)

    def memory_reserved(self, device_index=None):
        return torch.cuda.memory_reserved(device_index)

    def max_memory_reserved(self, device_index=None):
        return torch.cuda.max_memory_reserved(device_index)

    def reset_peak_memory_stats(self, device_index=None):
        return torch.cuda.reset_peak_memory_stats(device_index)

    def total_memory(self, device_index=None):
        return torch.cuda.get_device_properties(device_index or 0).total_memory

    def available_memory(self, device_index=None):
        free, _ = torch.cuda.mem_get_info(device_index)
        return free

    def memory_stats(self, device_index=None):
        return torch.cuda.memory_stats(device_index)

    # tracing: torch.cuda.nvtx is routed to roctx on ROCm, so rocprofv3 --marker-trace sees the ranges
    def range_push(self, msg):
        if os.environ.get("DS_ROCTX", "1") != "0":
            torch.cuda.nvtx.range_push(msg)

    def range_pop(self):
        if os.environ.get("DS_ROCTX", "1") != "0":
            torch.cuda.nvtx.range_pop()

    # graphs (hipGraph)
    def create_graph(self):
        return torch.cuda.CUDAGraph()

    def capture_to_graph(self, graph, pool=None, stream=None):
        return torch.cuda.graph(graph, pool, stream)

    def replay_graph(self, graph):
        graph.replay()

    def pin_memory(self, tensor, align_bytes=1):
        return tensor.pin_memory()

    def is_pinned(self, tensor):
        return tensor.is_pinned()

    def arch_name(self):
        return torch.cuda.get_device_properties(self.current_device()).gcnArchName.split(":")[0]


class _HostStream:
    """Stand-in for a device stream on the host path: everything is synchronous."""

    def __init__(self, *a, **k):
        pass

    def wait_stream(self, other):
        pass

    def wait_event(self, ev):
        pass

    def synchronize(self):
        pass

    def record_event(self, ev=None):
        return ev or _HostEvent()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _HostEvent:

    def __init__(self, enable_timing=False, **k):
        self.t = None

    def record(self, stream=None):
        import time
        self.t = time.perf_counter()

    def synchronize(self):
        pass

    def query(self):
        return True

    def wait(self, stream=None):
        pass

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class CpuAccelerator(_Base):
    """Host path used for gloo plumbing tests (BASELINE config 1). Not a performance target."""
    _name = "cpu"
    _comm = "gloo"

    def is_available(self):
        return True

    def device_count(self):
        return 1

    def current_device(self):
        return 0

    def device_name(self, device_index=None):
        return "cpu"

    def set_device(self, device_index):
        pass

    def synchronize(self, device_index=None):
        pass

    def manual_seed(self, seed):
        torch.manual_seed(seed)

    def manual_seed_all(self, seed):
        torch.manual_seed(seed)

    def get_rng_state(self, device_index=None):
        return torch.get_rng_state()

    def set_rng_state(self, new_state, device_index=None):
        torch.set_rng_state(new_state)

    def initial_seed(self):
        return torch.initial_seed()

    def default_generator(self, device_index):
        return torch.default_generator

    Stream = _HostStream
    Event = _HostEvent

    def stream(self, stream):
        return _HostStream()

    def current_stream(self, device_index=None):
        return _HostStream()

    def default_stream(self, device_index=None):
        return _HostStream()

    def empty_cache(self):
        pass

    def memory_allocated(self, device_index=None):
        return 0

    def max_memory_allocated(self, device_index=None):
        return 0

    def reset_max_memory_allocated(self, device_index=None):
        pass

    def memory_reserved(self, device_index=None):
        return 0

    def max_memory_reserved(self, device_index=None):
        return 0

    def reset_peak_memory_stats(self, device_index=None):
        pass

    def total_memory(self, device_index=None):
        import psutil
        return psutil.virtual_memory().total

    def available_memory(self, device_index=None):
        import psutil
        return psutil.virtual_memory().available

    def memory_stats(self, device_index=None):
        return {}

    def is_fp16_supported(self):
        return False

    def create_graph(self):
        return None

    def capture_to_graph(self, graph, pool=None, stream=None):
        import contextlib
        return contextlib.nullcontext()

    def replay_graph(self, graph):
        pass

    def pin_memory(self, tensor, align_bytes=1):
        return tensor

    def is_pinned(self, tensor):
        return False

    def arch_name(self):
        return "cpu"


_ACCEL = None


def get_accelerator():
    """Return the process-wide device facade (ROCm if a HIP device is visible, else host)."""
    global _ACCEL
    if _ACCEL is None:
        forced = os.environ.get("DS_ACCELERATOR", "").lower()
        if forced == "cpu":
            _ACCEL = CpuAccelerator()
        elif forced in ("cuda", "rocm", "hip"):
            _ACCEL = RocmAccelerator()
        else:
            _ACCEL = RocmAccelerator() if torch.cuda.is_available() else CpuAccelerator()
    return _ACCEL


def set_accelerator(accel):
    global _ACCEL
    _ACCEL = accel


@functools.lru_cache(None)
def is_rocm_device():
    return isinstance(get_accelerator(), RocmAccelerator)


# `deepspeed.accelerator.real_accelerator` is a sub-module path in the reference; this one-file accelerator answers it
# through the package's import-path finder, for which the module must look like a package
__path__ = []
