"""Loading a universal checkpoint into a live flat ZeRO optimizer (reference `checkpoint/universal_checkpoint.py:12-98`
`load_hp_checkpoint_state`, driven per parameter by `runtime/zero/stage_1_and_2.py:2213-2231` / `bf16_optimizer.py`).

Every rank reads each parameter's files (`<folder>/zero/<name>/{fp32,exp_avg,exp_avg_sq}.pt`), cuts out its
tensor-parallel slice by the recorded merge rule (the inverse of `ds_to_universal.merge_tp_slices`), and copies the
elements its own partition owns into the flat fp32 master / moment buffers and 16-bit shard
(`FlatZeroOptimizer._scatter_param`). No collective runs per parameter; the full 16-bit buffers of persistent groups
are refreshed once at the end.
"""
import os
import types

import torch

from . import constants as CK


def _safe(name):
    return name.replace("/", "_")


def tp_slice(entry, target_shape, tp_rank, tp_world_size):
    """This tensor-parallel rank's slice of a universal-checkpoint entry, shaped like the live parameter."""
    full = entry[CK.PARAM] if isinstance(entry, dict) else entry
    meta = entry if isinstance(entry, dict) else {}
    target_shape = tuple(target_shape)
    if tuple(full.shape) == target_shape:  # replicated / averaged parameters are stored whole
        return full
    if meta.get(CK.VOCAB_TENSOR, False):
        rows = target_shape[0] * tp_world_size
        if rows < full.shape[0]:
            raise ValueError(f"vocabulary tensor: padded size {rows} < universal size {full.shape[0]}")
        if rows > full.shape[0]:
            full = torch.nn.functional.pad(full, (0, 0, 0, rows - full.shape[0]))
    dim = meta.get(CK.CAT_DIM, 0)
    nsub = meta.get(CK.PARAM_N_SUB_PARAMS, 1)
    if nsub > 1:
        out = torch.cat([s.chunk(tp_world_size, dim=dim)[tp_rank] for s in full.chunk(nsub, dim=dim)], dim=dim)
    else:
        out = full.chunk(tp_world_size, dim)[tp_rank]
    if out.numel() != int(torch.Size(target_shape).numel()):
        raise ValueError(f"universal entry of shape {tuple(full.shape)} does not split into {tp_world_size} slices of "
                         f"{target_shape}")
    return out.reshape(target_shape)


@torch.no_grad()
def load_universal_into(optimizer, module, folder, tp_rank=0, tp_world_size=1, strict=True):
    """Scatter a universal checkpoint into the flat ZeRO optimizer of `module` (every rank calls this)."""
    from .zero_checkpoint import global_param_names
    zdir = os.path.join(folder, "zero")
    meta = torch.load(os.path.join(zdir, "optimizer_state.pt"), weights_only=True)
    gnames = global_param_names(module)
    names = {id(p): n for n, p in module.named_parameters()}
    ensured = False
    missing = []
    for p in optimizer.opt_params:
        local = names.get(id(p))
        if local is None:
            continue
        d = os.path.join(zdir, _safe(gnames.get(local, local)))
        f32 = os.path.join(d, "fp32.pt")
        if not os.path.isfile(f32):
            missing.append(local)
            continue
        shape = getattr(p, "ds_shape", p.shape)
        entry = torch.load(f32, weights_only=True, mmap=True)
        optimizer._scatter_param(p, tp_slice(entry, shape, tp_rank, tp_world_size), "fp32", also_shard=True)
        for key in ("exp_avg", "exp_avg_sq"):
            f = os.path.join(d, f"{key}.pt")
            if os.path.isfile(f):
                if not ensured:
                    optimizer._ensure_state()
                    ensured = True
                entry = torch.load(f, weights_only=True, mmap=True)
                optimizer._scatter_param(p, tp_slice(entry, shape, tp_rank, tp_world_size), key)
    if strict and missing:
        raise KeyError(f"universal checkpoint {folder} has no entry for {len(missing)} parameter(s), e.g. {missing[:3]}")
    if ensured:
        optimizer.set_step(int(meta.get("step", 0)))
    optimizer._post_step_gather()
    return meta


def load_hp_checkpoint_state(self, folder, tp_rank, tp_world_size):
    """Per-parameter entry point with the reference's signature: `param.load_hp_checkpoint_state(folder, tp_rank,
    tp_world_size)` with `folder` the parameter's own directory."""
    opt = self._ds_universal_optimizer
    shape = getattr(self, "ds_shape", self.shape)
    for key in ("fp32", "exp_avg", "exp_avg_sq"):
        f = os.path.join(folder, f"{key}.pt")
        if not os.path.isfile(f):
            if key == "fp32":
                raise FileNotFoundError(f"{f} is not a valid file")
            continue
        if key != "fp32":
            opt._ensure_state()
        entry = torch.load(f, weights_only=True, mmap=True)
        opt._scatter_param(self, tp_slice(entry, shape, tp_rank, tp_world_size), key, also_shard=key == "fp32")


def enable_universal_checkpoint(param_list, optimizer=None):
    for param in param_list:
        param._ds_universal_optimizer = optimizer
        param.load_hp_checkpoint_state = types.MethodType(load_hp_checkpoint_state, param)
