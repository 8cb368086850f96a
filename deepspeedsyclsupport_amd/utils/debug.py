"""Debug helpers (reference `utils/debug.py`): module / parameter names for log lines, a file-locked print that
keeps multi-rank output lines whole, per-rank log files, and a backward-graph walker."""
import fcntl
import os

module_names = {}
param_names = {}


def debug_clear_module_and_param_names():
    module_names.clear()
    param_names.clear()


def debug_extract_module_and_param_names(model):
    """Remember every module's and parameter's qualified name (call once, right after building the model)."""
    module_names.update({m: n for n, m in model.named_modules()})
    param_names.update({p: n for n, p in model.named_parameters()})


def debug_module2name(module):
    return module_names.get(module, "unknown")


def debug_module2name_id(module):
    return f"name={debug_module2name(module)} id={getattr(module, 'id', None)}"


def debug_module2name_class(module):
    return f"name={debug_module2name(module)} {module.__class__.__name__}"


def debug_param2name(param):
    return param_names.get(param, "unknown")


def debug_param2name_id(param):
    return f"name={debug_param2name(param)} id={getattr(param, 'ds_id', None)}"


def debug_param2name_id_shape(param):
    return f"{debug_param2name_id(param)} shape={tuple(getattr(param, 'ds_shape', param.shape))}"


def debug_param2name_id_shape_device(param):
    return f"{debug_param2name_id_shape(param)} device={param.device}"


def debug_param2name_id_numel(param):
    return f"{debug_param2name_id(param)} numel={getattr(param, 'ds_numel', param.numel())}"


def debug_param2name_id_shape_status(param):
    return f"{debug_param2name_id_shape(param)} status={getattr(param, 'ds_status', None)}"


def printflock(*msgs):
    """print() under an exclusive lock on this file, so lines from several ranks never interleave."""
    with open(__file__, "r") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            print(*msgs, flush=True)
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)


_rank_fh = None


def log_rank_file(rank, *msgs):
    """Append msgs to log_rank_<rank>.txt (diff two ranks' files to find where they diverge)."""
    global _rank_fh
    if _rank_fh is None:
        _rank_fh = open(f"log_rank_{rank}.txt", "w")
    for m in msgs:
        _rank_fh.write(f"{m}\n")
    _rank_fh.flush()


def print_backward_tensors(tensor):
    """Walk the autograd graph behind `tensor`, printing every tensor input of every node."""

    def walk(fn, depth=0):
        if fn is None:
            return
        var = getattr(fn, "variable", None)
        if var is not None:
            print(f"{'  ' * depth}{fn.name()}: tensor shape={tuple(var.shape)} grad={var.grad is not None}")
        for nxt, _ in getattr(fn, "next_functions", ()):
            walk(nxt, depth + 1)

    if getattr(tensor, "grad_fn", None) is not None:
        walk(tensor.grad_fn)
