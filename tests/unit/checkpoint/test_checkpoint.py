"""Checkpoint save/load round trips (reference `tests/unit/checkpoint/test_zero_optimizer.py`,
`test_latest_checkpoint.py`, `test_tag_validation.py`) and zero_to_fp32 consolidation
(`tests/unit/checkpoint/test_convert_checkpoint.py` style: consolidated fp32 == engine's gathered fp32 masters).

Resume test: train K steps, save, build a FRESH engine, load, train K more steps; the losses and final weights must
match an uninterrupted 2K-step run exactly (same data order), which only holds if fp32 masters, Adam moments,
step counts and the LR scheduler all round-trip.
"""
import os

import pytest
import torch

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama

STEPS = 2


def _cfg(stage, dtype):
    c = base_config(stage=stage, lr=1e-2, dtype=dtype)
    c["scheduler"] = {"type": "WarmupLR", "params": {"warmup_min_lr": 0.0, "warmup_max_lr": 1e-2,
                                                    "warmup_num_steps": 3}}
    return c


def _train(eng, data, steps):
    out = []
    for s in range(steps):
        x = data[s]
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        out.append(float(loss))
    return out


def _resume_run(stage, dtype, ckpt_dir, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    rank = dist.get_rank()
    data = random_tokens(2 * STEPS, 2, 16, seed=7 + rank)
    # uninterrupted
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=_cfg(stage, dtype))
    ref_losses = _train(eng, data, 2 * STEPS)
    ref_w = {n: safe_get_full_fp32_param(p) for n, p in eng.module.named_parameters()}
    # interrupted: K steps, save, fresh engine, load, K steps
    eng1, _, _, _ = ds.initialize(model=tiny_llama(), config=_cfg(stage, dtype))
    l1 = _train(eng1, data[:STEPS], STEPS)
    eng1.save_checkpoint(ckpt_dir, tag="t1")
    half_w = {n: safe_get_full_fp32_param(p) for n, p in eng1.module.named_parameters()}
    half_m = {n: safe_get_full_optimizer_state(p, "exp_avg") for n, p in eng1.module.named_parameters()}
    eng2, _, _, _ = ds.initialize(model=tiny_llama(seed=99), config=_cfg(stage, dtype))
    path, client = eng2.load_checkpoint(ckpt_dir)
    assert path is not None and path.endswith("t1")
    assert eng2.global_steps == STEPS
    for n, p in eng2.module.named_parameters():
        torch.testing.assert_close(safe_get_full_fp32_param(p), half_w[n], rtol=0, atol=0)
        torch.testing.assert_close(safe_get_full_optimizer_state(p, "exp_avg"), half_m[n], rtol=0, atol=0)
    l2 = _train(eng2, data[STEPS:], STEPS)
    got_w = {n: safe_get_full_fp32_param(p) for n, p in eng2.module.named_parameters()}
    if rank == 0:
        torch.save({"ref": ref_losses, "got": l1 + l2, "ref_w": ref_w, "got_w": got_w, "half_w": half_w}, out)


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_resume_matches_uninterrupted(stage, dtype, tmp_path):
    out = str(tmp_path / "r.pt")
    ckpt = str(tmp_path / "ckpt")
    run_distributed(_resume_run, 2, stage, dtype, ckpt, out)
    r = torch.load(out, weights_only=True)
    assert r["got"] == pytest.approx(r["ref"], rel=1e-6, abs=1e-6)
    for n in r["ref_w"]:
        torch.testing.assert_close(r["got_w"][n], r["ref_w"][n], rtol=0, atol=0, msg=n)
    assert os.path.isfile(os.path.join(ckpt, "latest"))
    assert os.path.isfile(os.path.join(ckpt, "zero_to_fp32.py")) or stage == 0
    if stage > 0:
        # consolidate with the standalone script's API and compare with the engine's gathered fp32 masters
        from deepspeedsyclsupport_amd.utils.zero_to_fp32 import get_fp32_state_dict_from_zero_checkpoint
        sd = get_fp32_state_dict_from_zero_checkpoint(ckpt)
        for n, v in r["half_w"].items():
            torch.testing.assert_close(sd[n], v, rtol=0, atol=0, msg=n)


def test_zero_to_fp32_cli(tmp_path):
    """The copy placed next to the checkpoint runs as a script and writes a weights_only-loadable file."""
    import subprocess
    import sys
    ckpt = str(tmp_path / "ckpt")
    run_distributed(_save_only, 2, ckpt)
    out = str(tmp_path / "fp32.bin")
    subprocess.run([sys.executable, os.path.join(ckpt, "zero_to_fp32.py"), ckpt, out], check=True)
    sd = torch.load(out, weights_only=True)
    ref = torch.load(os.path.join(ckpt, "ref.pt"), weights_only=True)
    for k, v in ref.items():
        torch.testing.assert_close(sd[k], v, rtol=0, atol=0)


def _save_only(ckpt):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=_cfg(3, "bf16"))
    _train(eng, random_tokens(2, 2, 16, seed=3 + dist.get_rank()), 2)
    eng.save_checkpoint(ckpt)
    ref = {n: safe_get_full_fp32_param(p) for n, p in eng.module.named_parameters()}
    if dist.get_rank() == 0:
        torch.save(ref, os.path.join(ckpt, "ref.pt"))


def _tag_mismatch(ckpt):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    c = _cfg(1, "fp32")
    c["checkpoint"] = {"tag_validation": "FAIL"}
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=c)
    with pytest.raises(ValueError):
        eng.save_checkpoint(ckpt, tag=f"tag{dist.get_rank()}")


def test_tag_validation_fail(tmp_path):
    run_distributed(_tag_mismatch, 2, str(tmp_path / "c"))


def _universal_src(ckpt, out):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    eng, _, _, _ = ds.initialize(model=tiny_llama(), config=_cfg(3, "fp32"))
    _train(eng, random_tokens(2, 2, 16, seed=21 + dist.get_rank()), 2)
    eng.save_checkpoint(ckpt, tag="u")
    ref = {n: (safe_get_full_fp32_param(p), safe_get_full_optimizer_state(p, "exp_avg"),
               safe_get_full_optimizer_state(p, "exp_avg_sq")) for n, p in eng.module.named_parameters()}
    if dist.get_rank() == 0:
        torch.save(ref, out)


def _universal_dst(ckpt, ref_path):
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd.utils import safe_get_full_fp32_param, safe_get_full_optimizer_state
    c = _cfg(1, "fp32")
    c["checkpoint"] = {"load_universal": True}
    eng, _, _, _ = ds.initialize(model=tiny_llama(seed=7), config=c)
    eng.load_checkpoint(ckpt, tag="u_universal")
    ref = torch.load(ref_path, weights_only=True)
    for n, p in eng.module.named_parameters():
        torch.testing.assert_close(safe_get_full_fp32_param(p), ref[n][0], rtol=0, atol=0, msg=n)
        torch.testing.assert_close(safe_get_full_optimizer_state(p, "exp_avg"), ref[n][1], rtol=0, atol=0)
        torch.testing.assert_close(safe_get_full_optimizer_state(p, "exp_avg_sq"), ref[n][2], rtol=0, atol=0)
    assert eng.global_steps == 2
    _train(eng, random_tokens(1, 2, 16, seed=99), 1)  # and training continues


def test_universal_checkpoint_changes_topology(tmp_path):
    """ZeRO-3 on 2 ranks -> universal -> ZeRO-1 on 3 ranks with every fp32 master and moment intact."""
    from deepspeedsyclsupport_amd.checkpoint.ds_to_universal import ds_to_universal
    ckpt, ref = str(tmp_path / "ck"), str(tmp_path / "ref.pt")
    run_distributed(_universal_src, 2, ckpt, ref)
    ds_to_universal(os.path.join(ckpt, "u"), os.path.join(ckpt, "u_universal"))
    run_distributed(_universal_dst, 3, ckpt, ref)
