"""Reference-layout optimizer shards written next to the native ones (`checkpoint/reference_format.py`).

The reader in this file is a test-side re-implementation of the reference's consolidation rules
(`utils/zero_to_fp32.py:141-191` parse_optim_states, `:256-326` ZeRO-2 merge, `:350-444` ZeRO-3 merge) and of its
universal-checkpoint fragment walk (`checkpoint/ds_to_universal.py:87-121`: `param_slice_mappings` start / numel into
`single_partition_of_fp32_groups` and `base_optimizer_state`). It must rebuild every fp32 weight and Adam moment from
the files this framework writes. No file written by the reference itself ships with it: byte parity stays unpinned.
"""
import glob
import math
import os
import re

import pytest
import torch

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama


def _train_and_save(stage, save_dir, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    cfg = base_config(stage=stage, lr=1e-2, mb=2)
    cfg["checkpoint"] = {"write_reference_format": True}
    model = tiny_llama()
    decay = [p for n, p in model.named_parameters() if p.dim() >= 2]
    no_decay = [p for n, p in model.named_parameters() if p.dim() < 2]
    groups = [{"params": decay, "weight_decay": 0.1}, {"params": no_decay, "weight_decay": 0.0}]
    eng, _, _, _ = ds.initialize(model=model, model_parameters=groups, config=cfg)
    for x in random_tokens(2, 2, 16, seed=5 + dist.get_rank()):
        eng.backward(eng(x, labels=x))
        eng.step()
    eng.save_checkpoint(save_dir, tag="t")
    full = {}
    for n, p in eng.module.named_parameters():
        full[n] = {"fp32": safe_get_full_fp32_param(p), "exp_avg": safe_get_full_optimizer_state(p, "exp_avg"),
                   "exp_avg_sq": safe_get_full_optimizer_state(p, "exp_avg_sq")}
    if dist.get_rank() == 0:
        torch.save(full, out)


# ---- the reference's reader, re-implemented --------------------------------------------------------------------
def _ref_files(ckpt_dir):
    optim = sorted(glob.glob(os.path.join(ckpt_dir, "*_optim_states.pt")),
                   key=lambda f: int(re.search(r"zero_pp_rank_(\d+)", f).group(1)))
    model = sorted(glob.glob(os.path.join(ckpt_dir, "*_model_states.pt")))
    return optim, model


def _ref_consolidate(ckpt_dir):
    optim, model = _ref_files(ckpt_dir)
    sds = [torch.load(f, map_location="cpu", weights_only=False)["optimizer_state_dict"] for f in optim]
    ms = torch.load(model[0], map_location="cpu", weights_only=False)
    stage = sds[0]["zero_stage"]
    world = sds[0]["partition_count"]
    world = max(world) if isinstance(world, list) else world
    assert world == len(optim)
    param_shapes = ms["param_shapes"]
    assert isinstance(ms["shared_params"], dict) and "buffer_names" in ms
    out = {}
    if stage <= 2:
        groups = [[sd["single_partition_of_fp32_groups"][i] for sd in sds] for i in range(len(param_shapes))]
        for shapes, parts in zip(param_shapes, groups):
            flat = torch.cat(parts, 0)
            off = 0
            for name, shape in shapes.items():
                n = shape.numel()
                out[name] = flat.narrow(0, off, n).view(shape)
                off += n
            align = 2 * world
            assert math.ceil(off / align) * align == math.ceil(flat.numel() / align) * align
    else:
        flats = [torch.cat(sd["fp32_flat_groups"], 0) for sd in sds]
        shapes = {k: v for d in param_shapes for k, v in d.items()}
        off = 0
        for name, shape in shapes.items():
            n = shape.numel()
            pn = math.ceil(n / world)
            out[name] = torch.cat([flats[r].narrow(0, off, pn) for r in range(world)], 0).narrow(0, 0, n).view(shape)
            off += pn
        assert off * world == flats[0].numel() * world
    return out, stage, sds, ms


def _ref_fragments(sds, key):
    """ds_to_universal's walk: per rank and group, every mapped fragment of `key`, concatenated per parameter."""
    frags = {}
    for sd in sds:
        state = sd["base_optimizer_state"]["state"]
        for gi, mapping in enumerate(sd["param_slice_mappings"]):
            flat = sd["single_partition_of_fp32_groups"][gi] if key == "fp32" else state[gi][key]
            for name, fr in mapping.items():
                frags.setdefault(name, []).append(flat.narrow(0, fr["start"], fr["numel"]))
    return {n: torch.cat(v) for n, v in frags.items()}


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_reference_reader_consolidates_our_files(stage, tmp_path):
    save, out = str(tmp_path / "ck"), str(tmp_path / "full.pt")
    run_distributed(_train_and_save, 4, stage, save, out)
    want = torch.load(out, weights_only=True)
    ref_dir = os.path.join(save, "reference_format")
    with open(os.path.join(ref_dir, "latest")) as f:
        assert f.read().strip() == "t"
    got, st, sds, ms = _ref_consolidate(os.path.join(ref_dir, "t"))
    assert st == stage and len(ms["param_shapes"]) == 2  # decay / no-decay groups kept apart
    assert set(got) == set(want)
    for n in want:
        torch.testing.assert_close(got[n], want[n]["fp32"], rtol=0, atol=0, msg=n)
    if stage <= 2:
        for key in ("fp32", "exp_avg", "exp_avg_sq"):
            fr = _ref_fragments(sds, key)
            for n in want:
                torch.testing.assert_close(fr[n].view(want[n][key].shape), want[n][key], rtol=0, atol=0, msg=f"{n} {key}")
        assert sum(sd["group_paddings"][0] for sd in sds[:-1]) == 0
    else:
        # moments follow the fp32 layout inside the torch-optimizer state
        shapes = {k: v for d in ms["param_shapes"] for k, v in d.items()}
        for key in ("exp_avg", "exp_avg_sq"):
            flats = [torch.cat([sd["optimizer_state_dict"]["state"][g][key] for g in range(2)]) for sd in sds]
            off = 0
            for n, shape in shapes.items():
                pn = math.ceil(shape.numel() / 4)
                full = torch.cat([f.narrow(0, off, pn) for f in flats]).narrow(0, 0, shape.numel()).view(shape)
                torch.testing.assert_close(full, want[n][key], rtol=0, atol=0, msg=f"{n} {key}")
                off += pn


def _resume(stage, save, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    cfg = base_config(stage=stage, lr=1e-2, mb=2)
    model = tiny_llama()
    decay = [p for n, p in model.named_parameters() if p.dim() >= 2]
    no_decay = [p for n, p in model.named_parameters() if p.dim() < 2]
    eng, _, _, _ = ds.initialize(model=model, config=cfg, model_parameters=[
        {"params": decay, "weight_decay": 0.1}, {"params": no_decay, "weight_decay": 0.0}])
    eng.load_checkpoint(save, tag="t")
    losses = []
    for x in random_tokens(2, 2, 16, seed=99):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss.detach()))
    if dist.get_rank() == 0:
        torch.save(losses, out)


@pytest.mark.parametrize("stage", [2, 3])
def test_engine_resumes_from_reference_format_at_another_world_size(stage, tmp_path):
    """The files the exporter writes are read back by the engine's reference-format sources (world 4 -> 2) and give
    the same next-step losses as resuming from the native shards."""
    save, full = str(tmp_path / "ck"), str(tmp_path / "full.pt")
    run_distributed(_train_and_save, 4, stage, save, full)
    a, b = str(tmp_path / "a.pt"), str(tmp_path / "b.pt")
    run_distributed(_resume, 2, stage, save, a)
    run_distributed(_resume, 2, stage, os.path.join(save, "reference_format"), b)
    assert torch.load(a, weights_only=True) == pytest.approx(torch.load(b, weights_only=True), rel=1e-6)


def test_offline_export_to_other_world_size(tmp_path):
    from deepspeedsyclsupport_amd.checkpoint import reference_format as rf
    save, out = str(tmp_path / "ck"), str(tmp_path / "full.pt")
    run_distributed(_train_and_save, 2, 2, save, out)
    import shutil
    shutil.rmtree(os.path.join(save, "reference_format"))
    files = rf.export_checkpoint(save, "t", world=3)
    assert len(files) == 3
    got, _, _, _ = _ref_consolidate(os.path.join(save, "reference_format", "t"))
    want = torch.load(out, weights_only=True)
    for n in want:
        torch.testing.assert_close(got[n], want[n]["fp32"], rtol=0, atol=0, msg=n)
