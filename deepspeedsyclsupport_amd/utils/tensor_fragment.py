"""Per-parameter access to ZeRO-partitioned fp32 state (reference `utils/tensor_fragment.py:101-257`:
safe_get_full_fp32_param, safe_get_full_optimizer_state, safe_get_full_grad, their setters and local variants).

With the flat-group design a parameter's fp32 master / Adam moments live as runs inside per-optimizer-group flat
partitions; the owning `FlatZeroOptimizer` gathers (full_*) or slices (local_*) them. The full_* getters are
collective over the parameter's data-parallel group (every rank must call them).
"""


def _owner(param):
    ref = getattr(param, "_ds_zero_optimizer", None)
    return ref() if ref is not None else None


def safe_get_full_fp32_param(param):
    opt = _owner(param)
    if opt is None:
        return param.detach().float() if param.numel() else None
    return opt.get_full_fp32_param(param)


def safe_set_full_fp32_param(param, value):
    opt = _owner(param)
    if opt is None:
        param.data.copy_(value)
        return
    opt.set_full_fp32_param(param, value)


def safe_get_full_optimizer_state(param, optim_state_key):
    opt = _owner(param)
    return None if opt is None else opt.get_full_optimizer_state(param, optim_state_key)


def safe_set_full_optimizer_state(param, value, optim_state_key):
    opt = _owner(param)
    if opt is not None:
        opt.set_full_optimizer_state(param, value, optim_state_key)


def safe_get_full_grad(param):
    opt = _owner(param)
    if opt is None:
        return None if param.grad is None else param.grad.detach().float()
    return opt.get_full_grad(param)


def safe_get_local_fp32_param(param):
    opt = _owner(param)
    return param.detach().float().reshape(-1) if opt is None else opt.get_local_fp32_param(param)


def safe_get_local_optimizer_state(param, optim_state_key):
    opt = _owner(param)
    return None if opt is None else opt.get_local_optimizer_state(param, optim_state_key)


def safe_get_local_grad(param):
    full = safe_get_full_grad(param)
    return None if full is None else full.reshape(-1)


def safe_set_local_fp32_param(param, value):
    """Overwrite this rank's fragment of the fp32 master (and its 16-bit shard) of `param`; no collective."""
    opt = _owner(param)
    if opt is None:
        param.data.copy_(value.reshape(param.shape))
    else:
        opt.set_local_fp32_param(param, value)


def safe_set_local_optimizer_state(param, value, optim_state_key):
    opt = _owner(param)
    if opt is not None:
        opt.set_local_optimizer_state(param, value, optim_state_key)


# the reference binds these three as methods on each low-precision parameter (`link_hp_params`); as functions they
# take the parameter first
def get_full_hp_param(param, optim_state_key=None):
    return safe_get_full_fp32_param(param) if optim_state_key is None else \
        safe_get_full_optimizer_state(param, optim_state_key)


def set_full_hp_param(param, value, optim_state_key=None):
    if optim_state_key is None:
        safe_set_full_fp32_param(param, value)
    else:
        safe_set_full_optimizer_state(param, value, optim_state_key)


def get_full_hp_grad(param):
    return safe_get_full_grad(param)

