#!/usr/bin/env python3
"""Write a ZeRO checkpoint's optimizer state in the reference's own on-disk layout.

The engine's native shards follow the flat-group layout of `runtime/zero/flat_optimizer.py` (rank segments of
parameter-order flat buffers, described by `ds_flat_layout`). Tools written against the reference read a different
arrangement, reproduced here from the reference's save code:

  * ZeRO-1/2 (`runtime/zero/stage_1_and_2.py:296-392,2102-2146`): per optimizer param group the trainable parameters
    are flattened back to back, padded to a multiple of 2 * world, cut into `world` equal partitions; rank r's file
    holds partition r without the tail padding (`single_partition_of_fp32_groups`), the same slices of the Adam
    moments (`base_optimizer_state`), `param_slice_mappings` (name -> start / numel of the parameter's fragment inside
    the partition), `group_paddings`, `partition_count`, `zero_stage`.
  * ZeRO-3 (`stage3.py:2382-2395`, consolidation rule `utils/zero_to_fp32.py:350-444`): every parameter is cut into
    `world` pieces of ceil(numel / world) elements (zero padded); rank r's file holds piece r of every parameter,
    concatenated in `param_shapes` order (`fp32_flat_groups`, one tensor per param group) and the same layout of the
    moments inside `optimizer_state_dict`.
  * model states: `param_shapes` as a list with one ordered name -> shape dict per param group, `buffer_names`,
    `shared_params`, `frozen_param_shapes` / `frozen_param_fragments`, `ds_version`.

The conversion is a re-slicing of data that already sits in the native shards, so it needs no collective: every rank
(or one offline process) opens the native files memory-mapped, rebuilds one parameter at a time
(`zero_checkpoint.FlatLayoutSource`) and copies the slices its reference file owns. Host memory stays at one
parameter plus the output partition being filled.

Output goes to `<save_dir>/reference_format/<tag>/` (+ `latest`), so `<save_dir>/reference_format` is a checkpoint
directory in the reference's sense. Differences that remain (no reference-written file ships with the reference, so
byte parity is unpinned): `loss_scaler` is a plain dict of the scaler's fields rather than a pickled scaler object,
and `param_slice_mappings` values are `{"start", "numel"}` dicts rather than `fragment_address` tuples (both load
without importing any class). MoE expert groups (partitioned over expert-data-parallel ranks) are not exported.

    python -m deepspeedsyclsupport_amd.checkpoint.reference_format <save_dir> [--tag TAG] [--world N]
"""
import argparse
import math
import os
from collections import OrderedDict

import torch

from . import constants as CK
from . import zero_checkpoint as zc

KEYS = ("fp32", "exp_avg", "exp_avg_sq")
SUBDIR = "reference_format"


def _resolve_tag(save_dir, tag):
    if tag is None:
        with open(os.path.join(save_dir, "latest")) as f:
            tag = f.read().strip()
    return str(tag)


def _model_file(tag_dir):
    files = sorted(f for f in os.listdir(tag_dir) if f.endswith(CK.MODEL_FILE_SUFFIX) and "expert_" not in f)
    if not files:
        raise FileNotFoundError(f"no *{CK.MODEL_FILE_SUFFIX} in {tag_dir}")
    return os.path.join(tag_dir, files[0])


def group_shapes(model_state):
    """[OrderedDict name -> shape] per optimizer param group, from a model-states dict."""
    shapes = model_state.get(CK.PARAM_SHAPES)
    if shapes is None:
        raise ValueError("model states carry no param_shapes: not a ZeRO checkpoint")
    if isinstance(shapes, dict):
        shapes = [shapes]
    return [OrderedDict((k, tuple(v)) for k, v in d.items()) for d in shapes]


def zero12_partition(shapes, world, rank):
    """Geometry of one param group under the reference's ZeRO-1/2 flattening: (partition size, lean length of this
    rank's partition, padding of this rank, [(name, param offset in the group, numel)])."""
    items, off = [], 0
    for name, shape in shapes.items():
        n = int(math.prod(shape))
        items.append((name, off, n))
        off += n
    total = off
    align = 2 * world
    padded = (total + align - 1) // align * align
    psize = padded // world
    lo = rank * psize
    lean = max(0, min(total, lo + psize) - lo)
    padding = padded - total if rank == world - 1 else 0
    return psize, lean, padding, items


def _moe_guard(source):
    for st in source.states:
        for g in st[CK.FLAT_LAYOUT]:
            if g.get("moe_group"):
                raise NotImplementedError("reference-format export of MoE expert groups is not supported "
                                          "(expert shards are partitioned over expert-data-parallel ranks)")


def build_reference_shard(source, shapes, native_osd, stage, world, rank):
    """The `optimizer_state_dict` of rank `rank` (of `world`) in the reference layout. `source` answers per-parameter
    full tensors, `shapes` is the per-group name -> shape list, `native_osd` supplies the scalar fields."""
    have_moments = source.has_moments()
    n_groups = len(shapes)
    step = source.step() if have_moments else None
    base_groups = (native_osd.get(CK.BASE_OPTIMIZER_STATE) or {}).get("param_groups") or [{} for _ in range(n_groups)]
    flats = {k: [] for k in KEYS}
    mappings, paddings = [], []
    for gi, d in enumerate(shapes):
        if stage <= 2:
            psize, lean, padding, items = zero12_partition(d, world, rank)
            lo, hi = rank * psize, rank * psize + lean
            out = {k: torch.zeros(lean, dtype=torch.float32) for k in KEYS if k == "fp32" or have_moments}
            mapping = OrderedDict()
            for name, off, n in items:
                a, b = max(off, lo), min(off + n, hi)
                if a >= b:
                    continue
                mapping[name] = {"start": a - lo, "numel": b - a}
                for k, buf in out.items():
                    v = source.get(name, k)
                    if v is None:
                        if k == "fp32":
                            raise KeyError(f"native shards hold no fp32 master for '{name}'")
                        continue
                    buf[a - lo:b - lo].copy_(v.reshape(-1)[a - off:b - off])
                    del v
            mappings.append(mapping)
            paddings.append(padding)
        else:
            pieces = {k: [] for k in KEYS if k == "fp32" or have_moments}
            for name, shape in d.items():
                n = int(math.prod(shape))
                pn = math.ceil(n / world)
                a, b = min(rank * pn, n), min((rank + 1) * pn, n)
                for k, lst in pieces.items():
                    piece = torch.zeros(pn, dtype=torch.float32)
                    v = source.get(name, k) if b > a else None
                    if v is not None:
                        piece[:b - a].copy_(v.reshape(-1)[a:b])
                        del v
                    elif k == "fp32" and b > a:
                        raise KeyError(f"native shards hold no fp32 master for '{name}'")
                    lst.append(piece)
            out = {k: (torch.cat(lst) if lst else torch.zeros(0)) for k, lst in pieces.items()}
        for k in KEYS:
            flats[k].append(out.get(k))
    state = {}
    groups = []
    for gi in range(n_groups):
        hyper = {k: v for k, v in (base_groups[gi] if gi < len(base_groups) else {}).items() if k != "params"}
        hyper["params"] = [gi]
        groups.append(hyper)
        if have_moments and flats["exp_avg"][gi] is not None:
            state[gi] = {"step": step if step is not None else 0, "exp_avg": flats["exp_avg"][gi],
                         "exp_avg_sq": flats["exp_avg_sq"][gi]}
    torch_state = {"state": state, "param_groups": groups}
    osd = OrderedDict()
    osd[CK.LOSS_SCALER] = native_osd.get(CK.LOSS_SCALER)
    osd["dynamic_loss_scale"] = native_osd.get("dynamic_loss_scale", False)
    osd["overflow"] = native_osd.get("overflow", False)
    if stage <= 2:
        osd[CK.CLIP_GRAD] = native_osd.get(CK.CLIP_GRAD, 0.0)
        osd[CK.BASE_OPTIMIZER_STATE] = torch_state
        osd[CK.SINGLE_PARTITION_OF_FP32_GROUPS] = flats["fp32"]
        osd[CK.ZERO_STAGE] = int(stage)
        osd[CK.GROUP_PADDINGS] = paddings
        osd[CK.PARTITION_COUNT] = [world] * n_groups
        osd[CK.PARAM_SLICE_MAPPINGS] = mappings
    else:
        osd[CK.ZERO_STAGE] = 3
        osd[CK.PARTITION_COUNT] = world
        osd[CK.OPTIMIZER_STATE_DICT] = torch_state
        osd[CK.FP32_FLAT_GROUPS] = flats["fp32"]
    osd[CK.DS_VERSION] = native_osd.get(CK.DS_VERSION)
    return osd


def _zero_name(stage_prefix, rank, mp_rank):
    return f"{stage_prefix}{CK.ZERO_FILE_PREFIX}{rank}_mp_rank_{mp_rank:02d}{CK.OPTIM_FILE_SUFFIX}"


def export_rank(save_dir, tag, rank, world=None, mp_rank=0, source=None):
    """Write rank `rank`'s reference-format optimizer shard (and, for rank 0 / ZeRO-3 every rank, the model states)
    of checkpoint `save_dir/tag` under `save_dir/reference_format/tag`. Returns the written optimizer file."""
    tag_dir = os.path.join(save_dir, tag)
    native_files = zc.optim_files(tag_dir, mp_rank) or zc.optim_files(tag_dir)
    if not native_files:
        raise FileNotFoundError(f"no native ZeRO shards in {tag_dir}")
    if source is None:
        source = zc.FlatLayoutSource(native_files)
    _moe_guard(source)
    native_osd = source.states[0]
    stage = int(native_osd[CK.ZERO_STAGE])
    world = int(world or len(native_files))
    ms = zc.load_file(_model_file(tag_dir))
    shapes = group_shapes(ms)
    out_dir = os.path.join(save_dir, SUBDIR, tag)
    os.makedirs(out_dir, exist_ok=True)
    prefix = os.path.basename(native_files[0]).split(CK.ZERO_FILE_PREFIX)[0]  # "bf16_" / "fp16_" / ""
    osd = build_reference_shard(source, shapes, native_osd, stage, world, rank)
    zpath = os.path.join(out_dir, _zero_name(prefix, rank, mp_rank))
    torch.save({CK.OPTIMIZER_STATE_DICT: osd, "ds_config": None, CK.DS_VERSION: native_osd.get(CK.DS_VERSION)}, zpath)
    if stage >= 3 or rank == 0:
        module = ms.get("module") or {}
        if stage >= 3:
            # the reference's ZeRO-3 module entries are empty placeholders (weights live in the optimizer shards)
            names = {n for d in shapes for n in d}
            module = OrderedDict((k, (v.new_zeros(0) if k in names and torch.is_tensor(v) else v))
                                 for k, v in module.items())
            mname = f"{CK.ZERO_FILE_PREFIX}{rank}_mp_rank_{mp_rank:02d}{CK.MODEL_FILE_SUFFIX}"
        else:
            mname = f"{CK.MODEL_FILE_PREFIX}{mp_rank:02d}{CK.MODEL_FILE_SUFFIX}"
        out = dict(ms)
        out["module"] = module
        out[CK.PARAM_SHAPES] = [OrderedDict((k, torch.Size(v)) for k, v in d.items()) for d in shapes]
        out["shared_params"] = ms.get("shared_params") or {}
        out["dp_world_size"] = world
        torch.save(out, os.path.join(out_dir, mname))
    if rank == 0:
        with open(os.path.join(save_dir, SUBDIR, "latest"), "w") as f:
            f.write(tag)
    return zpath


def export_checkpoint(save_dir, tag=None, world=None, mp_rank=0):
    """Offline: write every rank's reference-format files of one checkpoint (optionally for another world size)."""
    tag = _resolve_tag(save_dir, tag)
    tag_dir = os.path.join(save_dir, tag)
    native_files = zc.optim_files(tag_dir, mp_rank) or zc.optim_files(tag_dir)
    source = zc.FlatLayoutSource(native_files)
    world = int(world or len(native_files))
    return [export_rank(save_dir, tag, r, world, mp_rank, source) for r in range(world)]


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("save_dir")
    ap.add_argument("--tag", default=None)
    ap.add_argument("--world", type=int, default=None, help="data-parallel size of the written files (default: saved)")
    ap.add_argument("--mp_rank", type=int, default=0)
    a = ap.parse_args()
    for f in export_checkpoint(a.save_dir, a.tag, a.world, a.mp_rank):
        print(f)


if __name__ == "__main__":
    main()
