"""Flops profiler (reference `profiling/flops_profiler/profiler.py:28-1244`: per-module flops / MACs / params /
latency, `get_model_profile`, engine integration at `profile_step`).

Instead of monkey-patching `torch.nn.functional` the way the reference does, counting runs under PyTorch's
dispatcher-level `FlopCounterMode` (every aten matmul / conv / SDPA kernel is counted exactly once, whichever Python
API produced it, including hipBLASLt GEMMs issued by our own modules), with its module tracker giving the per-module
breakdown. Module latency comes from forward pre/post hooks bracketed by device synchronisation. Fused HIP kernels
(norms, activations, RoPE, cross-entropy) are memory-bound and are not counted as flops, matching the reference's
convention of counting only matmul-class work for transformer blocks.
"""
import sys
import time
from collections import defaultdict

import torch
from torch.utils.flop_counter import FlopCounterMode

from ...accelerator import get_accelerator


def number_to_string(num, units=None, precision=2):
    if units is None:
        for u, s in ((1e12, "T"), (1e9, "G"), (1e6, "M"), (1e3, "K")):
            if abs(num) >= u:
                return f"{num / u:.{precision}f} {s}"
        return f"{num:.{precision}f} "
    scale = {"T": 1e12, "G": 1e9, "M": 1e6, "K": 1e3, "": 1}[units]
    return f"{num / scale:.{precision}f} {units}"


def flops_to_string(flops, units=None, precision=2):
    return number_to_string(flops, units, precision) + "FLOPS"


def macs_to_string(macs, units=None, precision=2):
    return number_to_string(macs, units, precision) + "MACs"


def params_to_string(params_num, units=None, precision=2):
    return number_to_string(params_num, units, precision).strip()


def duration_to_string(duration, units=None, precision=2):
    if units is None:
        if duration >= 1:
            return f"{duration:.{precision}f} s"
        if duration >= 1e-3:
            return f"{duration * 1e3:.{precision}f} ms"
        return f"{duration * 1e6:.{precision}f} us"
    return f"{duration:.{precision}f} {units}"


class FlopsProfiler:

    def __init__(self, model, ds_engine=None, recompute_fwd_factor=0.0):
        self.model = model
        self.ds_engine = ds_engine
        self.recompute_fwd_factor = recompute_fwd_factor
        self.started = False
        self.func_patched = False
        self._mode = None
        self._hooks = []
        self._durations = defaultdict(float)
        self._t0 = {}
        self._names = {}

    # ------------------------------------------------------------------------------------------ control
    def start_profile(self, ignore_list=None):
        self.reset_profile()
        ignore = tuple(ignore_list or ())
        acc = get_accelerator()
        for name, m in self.model.named_modules():
            if ignore and isinstance(m, ignore):
                continue
            self._names[id(m)] = name or self.model.__class__.__name__
            m._ds_flops_profiler = self

            def pre(mod, inp):
                acc.synchronize()
                self._t0[id(mod)] = time.perf_counter()

            def post(mod, inp, out):
                acc.synchronize()
                self._durations[id(mod)] += time.perf_counter() - self._t0.pop(id(mod), time.perf_counter())

            self._hooks.append(m.register_forward_pre_hook(pre))
            self._hooks.append(m.register_forward_hook(post))
        self._mode = FlopCounterMode(display=False)
        self._mode.__enter__()
        self.started = True

    def stop_profile(self):
        if self._mode is not None and self.started:
            self._mode.__exit__(None, None, None)
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.started = False

    def reset_profile(self):
        self._durations.clear()
        self._t0.clear()

    def end_profile(self):
        self.stop_profile()
        self._mode = None

    # ------------------------------------------------------------------------------------------ results
    def _module_flops(self):
        if self._mode is None:
            return {}
        return {k: sum(v.values()) for k, v in self._mode.get_flop_counts().items()}

    def get_total_flops(self, as_string=False):
        total = self._mode.get_total_flops() if self._mode is not None else 0
        total = total * (1 + self.recompute_fwd_factor) if self.recompute_fwd_factor else total
        return flops_to_string(total) if as_string else total

    def get_total_macs(self, as_string=False):
        macs = self.get_total_flops() / 2
        return macs_to_string(macs) if as_string else macs

    def get_total_duration(self, as_string=False):
        d = self._durations.get(id(self.model), 0.0)
        return duration_to_string(d) if as_string else d

    def get_total_params(self, as_string=False):
        n = sum(p.ds_numel if hasattr(p, "ds_numel") else p.numel() for p in self.model.parameters())
        return params_to_string(n) if as_string else n

    def print_model_profile(self, profile_step=1, module_depth=-1, top_modules=1, detailed=True, output_file=None):
        out = open(output_file, "w") if output_file else sys.stdout
        flops, dur = self.get_total_flops(), self.get_total_duration()
        w = lambda s="": print(s, file=out)  # noqa: E731
        w("\n-------------------------- DeepSpeed Flops Profiler --------------------------")
        w(f"Profile Summary at step {profile_step}:")
        if self.ds_engine is not None:
            w(f"world size:                                   {self.ds_engine.world_size}")
            w(f"batch size per GPU:                           {self.ds_engine.train_micro_batch_size_per_gpu()}")
        w(f"params per GPU:                               {self.get_total_params(True)}")
        w(f"fwd MACs per GPU:                             {self.get_total_macs(True)}")
        w(f"fwd flops per GPU:                            {flops_to_string(flops)}")
        w(f"fwd latency:                                  {duration_to_string(dur)}")
        if dur > 0:
            w(f"fwd FLOPS per GPU = fwd flops / fwd latency:  {flops_to_string(flops / dur)}")
        if detailed:
            per_mod = self._module_flops()
            w("\n----------------------------- Aggregated Profile per GPU -----------------------------")
            depth_groups = defaultdict(list)
            for name, f in per_mod.items():
                depth = name.count(".")
                if module_depth >= 0 and depth > module_depth:
                    continue
                depth_groups[depth].append((f, name))
            for depth in sorted(depth_groups):
                top = sorted(depth_groups[depth], reverse=True)[:max(top_modules, 1)]
                w(f"depth {depth}: " + ", ".join(f"{n}: {flops_to_string(f)}" for f, n in top))
            w("\n------------------------------ Detailed Profile per GPU ------------------------------")
            for name, f in sorted(per_mod.items()):
                w(f"{name}: {flops_to_string(f)}")
        w("------------------------------------------------------------------------------")
        if output_file:
            out.close()


def _aggregated(self, module_depth=-1, top_modules=1):
    """{depth: [(module name, flops, seconds)]}: the `top_modules` largest modules of every depth by FLOPs."""
    per_mod = self._module_flops()
    by_name = {self._names[i]: d for i, d in self._durations.items() if i in self._names}
    root = self.model.__class__.__name__
    groups = defaultdict(list)
    for name, f in per_mod.items():
        if name == "Global":
            continue
        depth = name.count(".")
        if module_depth >= 0 and depth > module_depth:
            continue
        short = name[len(root) + 1:] if name.startswith(root + ".") else name
        groups[depth].append((name, f, by_name.get(short, by_name.get(name, 0.0))))
    return {d: sorted(v, key=lambda r: -r[1])[:max(top_modules, 1)] for d, v in sorted(groups.items())}


def _print_model_aggregated_profile(self, module_depth=-1, top_modules=1):
    """Top modules per depth by FLOPs with their forward latency (reference `profiler.py:386-430`)."""
    for depth, rows in _aggregated(self, module_depth, top_modules).items():
        print(f"depth {depth}:")
        print("    flops   - " + ", ".join(f"{n}: {flops_to_string(f)}" for n, f, _ in rows))
        print("    latency - " + ", ".join(f"{n}: {duration_to_string(t)}" for n, _, t in rows))


FlopsProfiler.print_model_aggregated_profile = _print_model_aggregated_profile
FlopsProfiler.is_expert_tensor_parallelism_enabled = lambda self: any(
    getattr(m, "enable_expert_tensor_parallelism", False) for m in self.model.modules())


def get_model_profile(model, input_shape=None, args=None, kwargs=None, print_profile=True, detailed=True,
                      module_depth=-1, top_modules=1, warm_up=1, as_string=True, output_file=None, ignore_modules=None,
                      mode="forward"):
    """Profile one forward (or `generate`) of `model`: returns (flops, macs, params)."""
    args = list(args or [])
    kwargs = dict(kwargs or {})
    if input_shape is not None:
        dev = next(model.parameters()).device
        dt = torch.long if mode == "generate" else next(model.parameters()).dtype
        args = [torch.ones(input_shape, dtype=dt, device=dev)]
    prof = FlopsProfiler(model)
    fn = model.generate if mode == "generate" else model
    with torch.no_grad():
        for _ in range(warm_up):
            fn(*args, **kwargs)
        prof.start_profile(ignore_list=ignore_modules)
        fn(*args, **kwargs)
        prof.stop_profile()
    flops, macs, params = prof.get_total_flops(), prof.get_total_macs(), prof.get_total_params()
    if print_profile:
        prof.print_model_profile(profile_step=warm_up, module_depth=module_depth, top_modules=top_modules,
                                 detailed=detailed, output_file=output_file)
    prof.end_profile()
    if as_string:
        return flops_to_string(flops), macs_to_string(macs), params_to_string(params)
    return flops, macs, params


def bytes_to_string(num, units=None, precision=2):
    return number_to_string(num, units=units, precision=precision) + "B"


def _profiler_of(module):
    prof = getattr(module, "_ds_flops_profiler", None)
    if prof is None:
        raise ValueError("the module is not being profiled: start a FlopsProfiler on its model first")
    return prof


def get_module_flops(module):
    """Forward FLOPs recorded for `module` (its sub-modules included) by the active profiler."""
    prof = _profiler_of(module)
    name = prof._names.get(id(module))
    root = prof.model.__class__.__name__
    counts = prof._module_flops()    # keyed "<RootClass>.<qualified name>" (the root itself: "<RootClass>")
    return int(counts.get(name if module is prof.model else f"{root}.{name}", 0))


def get_module_macs(module):
    return get_module_flops(module) // 2


def get_module_duration(module):
    """Forward wall time of `module` in seconds (device-synchronised around the module)."""
    return float(_profiler_of(module)._durations.get(id(module), 0.0))
