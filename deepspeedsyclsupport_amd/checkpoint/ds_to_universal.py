#!/usr/bin/env python3
"""ZeRO checkpoint -> universal checkpoint (reference `checkpoint/ds_to_universal.py:286`,
`universal_checkpoint.py:12`).

A universal checkpoint stores every parameter's full fp32 master and Adam moments as separate files
(`<out>/zero/<param name>/{fp32,exp_avg,exp_avg_sq}.pt`) plus the optimizer step, independent of the data-parallel
degree / ZeRO stage / partitioning that produced it. An engine started with `"checkpoint": {"load_universal": true}`
re-partitions those tensors into whatever flat layout it has, so training resumes with moments intact on a
different number of GPUs.

    python -m deepspeedsyclsupport_amd.checkpoint.ds_to_universal --input_folder ckpt/global_step10 \
        --output_folder ckpt/global_step10_universal
"""
import argparse
import os
import shutil

import torch

from ..utils import zero_to_fp32 as z

UNIVERSAL_KEYS = ("fp32", "exp_avg", "exp_avg_sq")


def _safe(name):
    return name.replace("/", "_")


def ds_to_universal(input_folder, output_folder):
    states = z.load_optim_states(input_folder)
    step = 0
    base = states[0].get("base_optimizer_state") or {}
    for st in base.get("state", {}).values():
        if "step" in st:
            step = int(st["step"]) if not torch.is_tensor(st["step"]) else int(st["step"].item())
    os.makedirs(os.path.join(output_folder, "zero"), exist_ok=True)
    for key in UNIVERSAL_KEYS:
        for name, t in z._reassemble(states, key).items():
            d = os.path.join(output_folder, "zero", _safe(name))
            os.makedirs(d, exist_ok=True)
            torch.save(t, os.path.join(d, f"{key}.pt"))
    torch.save({"step": step, "universal_checkpoint_version": 0.2}, os.path.join(output_folder, "zero",
                                                                                 "optimizer_state.pt"))
    # model-state files (module buffers, lr scheduler, counters) are carried over unchanged
    model_files = sorted(f for f in os.listdir(input_folder) if f.endswith(z.MODEL_FILE_SUFFIX))
    for f in model_files:
        shutil.copy(os.path.join(input_folder, f), os.path.join(output_folder, f))
    canonical = "mp_rank_00" + z.MODEL_FILE_SUFFIX  # what a non-ZeRO-3 engine looks for
    if model_files and canonical not in model_files:
        shutil.copy(os.path.join(input_folder, model_files[0]), os.path.join(output_folder, canonical))
    return output_folder


def load_universal_into(optimizer, module, folder):
    """Scatter a universal checkpoint into the flat ZeRO optimizer of `module` (every rank calls this)."""
    zdir = os.path.join(folder, "zero")
    meta = torch.load(os.path.join(zdir, "optimizer_state.pt"), weights_only=True)
    for name, p in module.named_parameters():
        d = os.path.join(zdir, _safe(name))
        if not os.path.isdir(d) or id(p) not in optimizer.param_group:
            continue
        dev = optimizer.device
        optimizer.set_full_fp32_param(p, torch.load(os.path.join(d, "fp32.pt"), weights_only=True).to(dev))
        for key in ("exp_avg", "exp_avg_sq"):
            f = os.path.join(d, f"{key}.pt")
            if os.path.exists(f):
                optimizer._ensure_state(key)
                optimizer.set_full_optimizer_state(p, torch.load(f, weights_only=True).to(dev), key)
    optimizer.set_step(meta["step"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--input_folder", required=True)
    ap.add_argument("--output_folder", required=True)
    ap.add_argument("--num_extract_workers", type=int, default=4)
    ap.add_argument("--num_merge_workers", type=int, default=2)
    a = ap.parse_args()
    ds_to_universal(a.input_folder, a.output_folder)


if __name__ == "__main__":
    main()
