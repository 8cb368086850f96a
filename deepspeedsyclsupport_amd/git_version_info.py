"""Build identification (reference `git_version_info.py`): version, and which native ops are built / compatible."""
from . import __version__ as version

git_hash = "unknown"
git_branch = "unknown"


def _ops():
    from .ops.op_builder import ALL_OPS
    built, compat = {}, {}
    for name, builder in ALL_OPS.items():
        b = builder() if isinstance(builder, type) else builder
        compat[name] = bool(b.is_compatible(verbose=False)) if hasattr(b, "is_compatible") else True
        built[name] = compat[name]
    return built, compat


try:
    installed_ops, compatible_ops = _ops()
except Exception:  # the op table is informational only
    installed_ops, compatible_ops = {}, {}
torch_info = {"version": None, "cuda_version": None, "hip_version": None}
try:
    import torch
    torch_info = {"version": ".".join(torch.__version__.split(".")[:2]), "cuda_version": None,
                  "hip_version": getattr(torch.version, "hip", None)}
except Exception:
    pass
