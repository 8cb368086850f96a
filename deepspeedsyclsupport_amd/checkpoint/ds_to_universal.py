#!/usr/bin/env python3
"""ZeRO checkpoint -> universal checkpoint, one parameter at a time (reference `checkpoint/ds_to_universal.py:87-319`).

A universal checkpoint stores every parameter's full fp32 master and Adam moments as separate files
(`<out>/zero/<param name>/{fp32,exp_avg,exp_avg_sq}.pt`, each `{"param": tensor, "cat_dim": ..., "vocab_tensor":
..., "param_n_sub_params": ...}` as the reference writes them) plus `zero/optimizer_state.pt` with the unsharded
optimizer fields, independent of the data-parallel / tensor-parallel degree and ZeRO stage that produced it. An engine
started with `"checkpoint": {"load_universal": true}` re-partitions those tensors into whatever flat layout it has
(`universal_checkpoint.load_universal_into`).

The reference extracts every rank's fragments into a temp tree and merges them in a second pass with worker pools.
Here the shard files are opened memory-mapped (`zero_checkpoint.open_source`, which reads this framework's flat shards
and the reference's ZeRO-1/2/3 layouts alike) and each parameter is rebuilt, merged across tensor-parallel ranks and
written before the next one is touched: host memory holds the TP slices of ONE parameter plus their merge (about
twice the largest parameter), whatever the model size. `stats["peak_live_bytes"]` reports that bound as it was met.

Tensor-parallel slices (one source per `mp_rank_XX`) are merged by the rules the client recorded under
`universal_checkpoint_info` in its checkpoint state (reference `merge_tp_slices`, `ds_to_universal.py:156-221`):
replicated (first slice), averaged, two fused sub-parameters concatenated on dim 0 (e.g. gate|up), row-parallel
(concatenate on dim 1), default column-parallel (dim 0); vocabulary tensors drop their padding rows.

    python -m deepspeedsyclsupport_amd.checkpoint.ds_to_universal --input_folder ckpt/global_step10 \
        --output_folder ckpt/global_step10_universal
"""
import argparse
import os
import re
import shutil

import torch

from . import constants as CK
from . import zero_checkpoint as zc

UNIVERSAL_KEYS = ("fp32", "exp_avg", "exp_avg_sq")


def _safe(name):
    return name.replace("/", "_")


def _match(patterns, name, used):
    hit = [p for p in patterns if re.match(p, name)]
    if len(hit) > 1:
        raise ValueError(f"more than one pattern {hit} matches '{name}'")
    if hit:
        used.add(hit[0])
    return bool(hit)


def merge_tp_slices(name, slices, info, used):
    """-> the reference's per-file dict for one state of one parameter."""
    out = {}
    if _match(info.get(CK.TP_REPLICATED_PARAMETER_PATTERNS, []), name, used):
        if any(not torch.equal(slices[0], o) for o in slices[1:]):
            raise ValueError(f"'{name}' is declared replicated across tensor-parallel ranks but its slices differ")
        param = slices[0]
    elif _match(info.get(CK.PARAMETER_TO_AVERAGE_PATTERNS, []), name, used):
        param = sum(slices) / len(slices) if len(slices) > 1 else slices[0]
    elif _match(info.get(CK.PARAMETER_WITH_2_SUB_PARAMS_CAT_DIM_0, []), name, used):
        halves = [torch.chunk(s, 2, dim=0) for s in slices]
        param = torch.cat([h[0] for h in halves] + [h[1] for h in halves], dim=0) if len(slices) > 1 else slices[0]
        out[CK.CAT_DIM] = 0
        out[CK.PARAM_N_SUB_PARAMS] = 2
    else:
        dim = 1 if _match(info.get(CK.PARAMETER_WITH_ROW_PARALLELISM_PATTERNS, []), name, used) else 0
        param = torch.cat(slices, dim=dim) if len(slices) > 1 else slices[0]
        out[CK.CAT_DIM] = dim
    if _match(info.get(CK.VOCABULARY_PARAMETER_PATTERNS, []), name, used):
        param = param[:info[CK.ORIGINAL_VOCAB_SIZE]]
        out[CK.VOCAB_TENSOR] = True
    out[CK.PARAM] = param.contiguous()
    return out


def _mp_ranks(input_folder):
    ranks = sorted({zc._rank_of(f)[0] for f in zc.optim_files(input_folder)})
    return ranks or [0]


def ds_to_universal(input_folder, output_folder, strict=False):
    """Convert one checkpoint tag directory. Returns stats (parameters written, peak bytes held at once, largest
    parameter's bytes)."""
    mp_ranks = _mp_ranks(input_folder)
    sources = [zc.open_source(input_folder, mp) for mp in mp_ranks]
    model_files = sorted(f for f in os.listdir(input_folder) if f.endswith(CK.MODEL_FILE_SUFFIX) and "expert_" not in f)
    info = {}
    if model_files:
        ms = zc.load_file(os.path.join(input_folder, model_files[0]))
        info = ms.get(CK.UNIVERSAL_CHECKPOINT_INFO) or {}
    if len(sources) > 1 and not info:
        raise ValueError(f"{input_folder} holds {len(sources)} tensor-parallel ranks but its checkpoint state has no "
                         f"'{CK.UNIVERSAL_CHECKPOINT_INFO}' telling how their slices merge")
    zdir = os.path.join(output_folder, "zero")
    os.makedirs(zdir, exist_ok=True)
    used = set()
    stats = {"params": 0, "peak_live_bytes": 0, "largest_param_bytes": 0, "tp_degree": len(sources)}
    have_moments = sources[0].has_moments()
    for name in sources[0].names():
        d = os.path.join(zdir, _safe(name))
        os.makedirs(d, exist_ok=True)
        for key in UNIVERSAL_KEYS if have_moments else ("fp32", ):
            slices = []
            for s in sources:
                v = s.get(name, key)
                if v is not None:
                    slices.append(v)
            if not slices:
                continue
            held = sum(t.numel() * 4 for t in slices)
            entry = merge_tp_slices(name, slices, info, used)
            merged = entry[CK.PARAM]
            if len(slices) > 1 or merged.data_ptr() != slices[0].data_ptr():
                held += merged.numel() * 4
            stats["peak_live_bytes"] = max(stats["peak_live_bytes"], held)
            stats["largest_param_bytes"] = max(stats["largest_param_bytes"], merged.numel() * 4)
            torch.save(entry, os.path.join(d, f"{key}.pt"))
            del slices, entry, merged
        stats["params"] += 1
    patterns = {p for k in (CK.TP_REPLICATED_PARAMETER_PATTERNS, CK.PARAMETER_TO_AVERAGE_PATTERNS,
                            CK.PARAMETER_WITH_ROW_PARALLELISM_PATTERNS, CK.VOCABULARY_PARAMETER_PATTERNS,
                            CK.PARAMETER_WITH_2_SUB_PARAMS_CAT_DIM_0) for p in info.get(k, [])}
    unused = sorted(patterns - used)
    if unused and strict:
        raise ValueError(f"unused patterns while merging tensor-parallel slices: {unused}")
    stats["unused_patterns"] = unused
    # unsharded optimizer fields (reference `_save_optimizer_state`): everything but the sharded tensors
    osd = sources[0].states[0]
    sharded = (CK.BASE_OPTIMIZER_STATE, CK.PARAM_SLICE_MAPPINGS, CK.SINGLE_PARTITION_OF_FP32_GROUPS,
               CK.FP32_FLAT_GROUPS, CK.OPTIMIZER_STATE_DICT, CK.FLAT_LAYOUT, "fp32_host_partitions",
               "host_optimizer_states")
    common = {k: v for k, v in osd.items() if k not in sharded}
    common["step"] = int(sources[0].step() or 0)
    base = osd.get(CK.BASE_OPTIMIZER_STATE) or osd.get(CK.OPTIMIZER_STATE_DICT) or {}
    if isinstance(base, dict) and base.get("param_groups"):
        common["param_groups"] = [{k: v for k, v in g.items() if k != "params"} for g in base["param_groups"]]
    common[CK.UNIVERSAL_CHECKPOINT_VERSION_KEY] = CK.UNIVERSAL_CHECKPOINT_VERSION_VALUE
    torch.save(common, os.path.join(zdir, "optimizer_state.pt"))
    # model-state files (module buffers, lr scheduler, counters) are carried over unchanged
    for f in model_files:
        shutil.copy(os.path.join(input_folder, f), os.path.join(output_folder, f))
    canonical = CK.MODEL_FILE_PREFIX + "00" + CK.MODEL_FILE_SUFFIX  # what a non-ZeRO-3 engine looks for
    if model_files and canonical not in model_files:
        shutil.copy(os.path.join(input_folder, model_files[0]), os.path.join(output_folder, canonical))
    return stats


def load_universal_into(optimizer, module, folder, tp_rank=0, tp_world_size=1):
    from .universal_checkpoint import load_universal_into as impl
    return impl(optimizer, module, folder, tp_rank, tp_world_size)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--input_folder", required=True)
    ap.add_argument("--output_folder", required=True)
    ap.add_argument("--num_extract_workers", type=int, default=4, help="accepted for command-line parity; the "
                    "conversion streams one parameter at a time in this process")
    ap.add_argument("--num_merge_workers", type=int, default=2, help="accepted for command-line parity")
    ap.add_argument("--keep_temp_folder", action="store_true", help="accepted for command-line parity (no temp tree)")
    ap.add_argument("--strict", action="store_true", help="fail when a merge pattern matched no parameter")
    a = ap.parse_args()
    print(ds_to_universal(a.input_folder, a.output_folder, strict=a.strict))


if __name__ == "__main__":
    main()
