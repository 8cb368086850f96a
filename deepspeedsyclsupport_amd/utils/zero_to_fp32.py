#!/usr/bin/env python3
"""Consolidate a ZeRO checkpoint into one fp32 state_dict (reference `utils/zero_to_fp32.py:468-592`).

Standalone on purpose (the engine copies it next to every checkpoint): needs only torch.

    python zero_to_fp32.py <checkpoint_dir> <output_file> [-t TAG] [--safe_serialization]

Each rank's `*_optim_states.pt` holds its fp32 master partitions (`single_partition_of_fp32_groups`, one flat
tensor per optimizer group) plus a layout descriptor (`ds_flat_layout`): for every flat parameter group, the
per-rank segment size / offset, which slices ("runs") of the segment live in which optimizer-group master at which
offset (or in the host master for Twin-Flow / offload runs), and (name, shape, offset, numel) of every parameter.
Reassembly is per parameter over every rank's own layout, so MoE expert groups (partitioned over expert-data-
parallel ranks; expert-parallel ranks hold different experts, recorded under their global expert ids) and
model-parallel ranks (one rank's files at a time) come out right. Files are read with `torch.load(weights_only=True)`.

Format note: the flat-group shards are NOT the reference's per-group layout (`single_partition_of_fp32_groups`
sliced by `param_shapes`), so the reference's zero_to_fp32 cannot read them; this script can, and
`checkpoint/zero_checkpoint.py` reads both formats (the engine loads reference-format checkpoints through it).
`"checkpoint": {"write_reference_format": true}` (or `python -m deepspeedsyclsupport_amd.checkpoint.reference_format`
offline) additionally writes the reference's own layout under `<save_dir>/reference_format/<tag>` for tools written
against it.
"""
import argparse
import glob
import os
import re
from collections import OrderedDict

import torch

OPTIM_FILE_SUFFIX = "_optim_states.pt"
MODEL_FILE_SUFFIX = "_model_states.pt"
FLAT_LAYOUT = "ds_flat_layout"
SINGLE_PARTITION_OF_FP32_GROUPS = "single_partition_of_fp32_groups"
OPTIMIZER_STATE_DICT = "optimizer_state_dict"
BUFFER_NAMES = "buffer_names"


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def _rank_of(path):
    m = re.search(r"zero_pp_rank_(\d+)_mp_rank_(\d+)", os.path.basename(path))
    return (int(m.group(2)), int(m.group(1))) if m else (0, 0)


def get_optim_files(ckpt_dir, mp_rank=0):
    files = sorted((f for f in glob.glob(os.path.join(ckpt_dir, f"*{OPTIM_FILE_SUFFIX}")) if "zero_pp_rank_" in f),
                   key=_rank_of)
    if any(_rank_of(f)[0] == mp_rank for f in files):
        files = [f for f in files if _rank_of(f)[0] == mp_rank]  # one model-parallel rank's data-parallel shards
    if not files:
        raise FileNotFoundError(f"no *{OPTIM_FILE_SUFFIX} files in {ckpt_dir}")
    return files


def get_model_state_file(ckpt_dir):
    files = sorted(f for f in glob.glob(os.path.join(ckpt_dir, f"*{MODEL_FILE_SUFFIX}")) if "expert_" not in f)
    if not files:
        raise FileNotFoundError(f"no *{MODEL_FILE_SUFFIX} files in {ckpt_dir}")
    return files[0]


def _resolve(checkpoint_dir, tag):
    if tag is None:
        latest = os.path.join(checkpoint_dir, "latest")
        if not os.path.isfile(latest):
            raise ValueError(f"no 'latest' file in {checkpoint_dir}; pass tag explicitly")
        with open(latest) as f:
            tag = f.read().strip()
    path = os.path.join(checkpoint_dir, tag)
    if not os.path.isdir(path):
        raise FileNotFoundError(f"directory {path} does not exist")
    return path


def _flat_source(st, key):
    """fetch(og, on_host) -> the rank's flat fp32 tensor holding `key` (fp32 master or an Adam moment)."""
    masters = st[SINGLE_PARTITION_OF_FP32_GROUPS]
    host = st.get("fp32_host_partitions") or []
    base = st.get("base_optimizer_state") or {}
    host_states = st.get("host_optimizer_states") or {}
    idx = {"exp_avg": 0, "exp_avg_sq": 1}

    def fetch(og, on_host):
        if key == "fp32":
            return host[og] if on_host else masters[og]
        if on_host:
            hs = host_states.get(og, host_states.get(str(og)))
            return None if hs is None else hs[idx[key]]
        pid = base["param_groups"][og]["params"][0]
        return base["state"].get(pid, {}).get(key)

    return fetch


def _reassemble(states, key):
    """Per-parameter reassembly from EVERY rank's own layout (groups may differ per rank: MoE expert groups are
    partitioned over expert-data-parallel ranks and expert-parallel ranks hold different experts, so expert parameters
    are keyed by their GLOBAL name). Raises when the ranks' shards do not cover a parameter completely."""
    index = OrderedDict()
    for r, st in enumerate(states):
        for g in st[FLAT_LAYOUT]:
            gn = g.get("global_names") or {}
            for (name, shape, off, numel) in g["params"]:
                index.setdefault(gn.get(name, name), []).append((r, g, tuple(shape), off, numel))
    out = OrderedDict()
    for name, ents in index.items():
        shape, numel = ents[0][2], ents[0][4]
        buf = torch.zeros(numel, dtype=torch.float32)
        cov = torch.zeros(numel, dtype=torch.bool)
        for (r, g, _, off, _) in ents:
            fetch = _flat_source(states[r], key)
            lo = g["seg_lo"]
            for (s, e, og, moff, on_host) in g["runs"]:
                a, b = max(lo + s, off), min(lo + e, off + numel)
                if a >= b:
                    continue
                src = fetch(og, on_host)
                if src is None:
                    continue
                buf[a - off:b - off] = src[moff + a - lo - s:moff + b - lo - s].float()
                cov[a - off:b - off] = True
        if not bool(cov.all()):
            raise ValueError(f"'{name}': the {len(states)} shard files cover {int(cov.sum())}/{numel} elements "
                             f"(missing rank files?)")
        out[name] = buf.view(shape)
    return out


def _reassemble_frozen(states):
    """Frozen parameters ZeRO-3 partitioned without optimizer state: name -> full fp32 tensor, cut out of every
    rank's `frozen_shards` by its `frozen_layout` (segment geometry + per-parameter offsets)."""
    index = OrderedDict()
    for r, st in enumerate(states):
        for gi, g in enumerate(st.get("frozen_layout") or []):
            for (name, shape, off, numel) in g["params"]:
                index.setdefault(name, []).append((r, gi, g, tuple(shape), off, numel))
    out = OrderedDict()
    for name, ents in index.items():
        shape, numel = ents[0][3], ents[0][5]
        buf = torch.zeros(numel, dtype=torch.float32)
        cov = torch.zeros(numel, dtype=torch.bool)
        for (r, gi, g, _, off, _) in ents:
            shard = states[r]["frozen_shards"][gi]
            lo = g["seg_lo"]
            a, b = max(lo, off), min(lo + g["seg"], off + numel)
            if a < b:
                buf[a - off:b - off] = shard[a - lo:b - lo].float()
                cov[a - off:b - off] = True
        if not bool(cov.all()):
            raise ValueError(f"frozen '{name}': the {len(states)} shard files cover {int(cov.sum())}/{numel} elements")
        out[name] = buf.view(shape)
    return out


def load_optim_states(ds_checkpoint_dir):
    return [_load(f)[OPTIMIZER_STATE_DICT] for f in get_optim_files(ds_checkpoint_dir)]


def _get_fp32_state_dict_from_zero_checkpoint(ds_checkpoint_dir, exclude_frozen_parameters=False):
    states = load_optim_states(ds_checkpoint_dir)
    out = _reassemble(states, "fp32")
    if not exclude_frozen_parameters:
        out.update(_reassemble_frozen(states))
    # non-expert parameters whose 16-bit placeholders are empty (ZeRO-3) come only from the shards above
    # buffers (and any non-partitioned tensors) come from the 16-bit model file
    try:
        model_sd = _load(get_model_state_file(ds_checkpoint_dir))
        buffers = set(model_sd.get(BUFFER_NAMES, []) or [])
        for k, v in (model_sd.get("module") or {}).items():
            if torch.is_tensor(v) and v.numel() == 0:
                continue  # partitioned placeholder
            if k in buffers or (k not in out and not exclude_frozen_parameters):
                out[k] = v.float() if torch.is_floating_point(v) else v
    except FileNotFoundError:
        pass
    return out


def get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag=None, exclude_frozen_parameters=False):
    return _get_fp32_state_dict_from_zero_checkpoint(_resolve(checkpoint_dir, tag), exclude_frozen_parameters)


def convert_zero_checkpoint_to_fp32_state_dict(checkpoint_dir, output_file, tag=None,
                                               exclude_frozen_parameters=False, safe_serialization=False):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag, exclude_frozen_parameters)
    if safe_serialization:
        from safetensors.torch import save_file
        save_file({k: v.contiguous() for k, v in sd.items()}, output_file)
    else:
        torch.save(sd, output_file)
    return sd


def load_state_dict_from_zero_checkpoint(model, checkpoint_dir, tag=None):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag)
    model = model.cpu()
    model.load_state_dict(sd, strict=False)
    return model


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("checkpoint_dir")
    ap.add_argument("output_file")
    ap.add_argument("-t", "--tag", default=None)
    ap.add_argument("--exclude_frozen_parameters", action="store_true")
    ap.add_argument("--safe_serialization", action="store_true")
    a = ap.parse_args()
    convert_zero_checkpoint_to_fp32_state_dict(a.checkpoint_dir, a.output_file, a.tag, a.exclude_frozen_parameters,
                                               a.safe_serialization)


# ---- file discovery helpers with the reference's names
def atoi(text):
    return int(text) if text.isdigit() else text


def natural_keys(text):
    """Sort key that orders "rank_2" before "rank_10"."""
    import re
    return [atoi(c) for c in re.split(r"(\d+)", text)]


def get_checkpoint_files(checkpoint_dir, glob_pattern):
    import glob
    files = sorted(glob.glob(os.path.join(checkpoint_dir, glob_pattern)), key=natural_keys)
    if not files:
        raise FileNotFoundError(f"can't find {glob_pattern} files in directory '{checkpoint_dir}'")
    return files


def get_model_state_files(checkpoint_dir):
    return get_checkpoint_files(checkpoint_dir, "*_model_states.pt")

