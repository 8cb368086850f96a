"""Autotuner (reference `tests/unit/autotuning/test_autotuning.py`): memory-model pruning, candidate generation,
best-config selection (fake experiments), and one real end-to-end tuning run of a tiny script through the launcher."""
import json
import os
import subprocess
import sys
import types

import pytest

from deepspeedsyclsupport_amd.autotuning import Autotuner

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _args(user_args):
    return types.SimpleNamespace(user_script="train.py", user_args=user_args)


def test_memory_model_and_selection(tmp_path):
    base = {"train_micro_batch_size_per_gpu": 1, "autotuning": {
        "enabled": True, "results_dir": str(tmp_path / "res"), "exps_dir": str(tmp_path / "exps"),
        "max_train_micro_batch_size_per_gpu": 16, "num_tuning_micro_batch_sizes": 3,
        "activation_mem_per_sample": 2 * 1024**3}}
    seen = []

    def fake(exp):
        seen.append((exp["stage"], exp["mbs"]))
        # throughput rises with mbs, ZeRO-3 pays a 10% comm tax
        return {"throughput": exp["mbs"] * (0.9 if exp["stage"] == 3 else 1.0)}

    # 7B params on 8 GPUs with 64 GB devices: unpartitioned stage-0 states (16 B/param) do not fit
    at = Autotuner(_args([]), {"localhost": list(range(8))}, base_config=base, run_experiment=fake,
                   gpu_mem_bytes=64 * 1024**3, num_params=7e9)
    assert at.max_mbs_for(0) == 0 and at.max_mbs_for(3) > 0
    best = at.tune()
    assert all(st >= 1 for st, _ in seen), seen
    assert best[0]["stage"] == 2 and best[0]["mbs"] == max(m for s, m in seen if s == 2)
    opt = json.load(open(tmp_path / "res" / "ds_config_optimal.json"))
    assert opt["zero_optimization"]["stage"] == 2 and "autotuning" not in opt


def test_autotuning_end_to_end(tmp_path):
    script = tmp_path / "train.py"
    script.write_text(
        "import argparse, json, sys, torch\n"
        f"sys.path.insert(0, {REPO!r}); sys.path.insert(0, {os.path.join(REPO, 'tests')!r})\n"
        "import deepspeedsyclsupport_amd as ds\n"
        "from unit.simple_model import tiny_llama, random_tokens\n"
        "p = argparse.ArgumentParser(); p.add_argument('--local_rank', type=int, default=0)\n"
        "p.add_argument('--deepspeed_config'); a = p.parse_args()\n"
        "eng, _, _, _ = ds.initialize(model=tiny_llama(), config=a.deepspeed_config)\n"
        "mb = eng.train_micro_batch_size_per_gpu()\n"
        "for x in random_tokens(50, mb, 16):\n"
        "    loss = eng(x, labels=x); eng.backward(loss); eng.step()\n")
    cfg = {"train_micro_batch_size_per_gpu": 1, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           "autotuning": {"enabled": True, "results_dir": str(tmp_path / "res"), "exps_dir": str(tmp_path / "exps"),
                          "zero_stages": [0, 3], "max_train_micro_batch_size_per_gpu": 2,
                          "num_tuning_micro_batch_sizes": 2, "start_profile_step": 1, "end_profile_step": 2}}
    cfg_path = tmp_path / "ds.json"
    cfg_path.write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=REPO, DS_ACCELERATOR="cpu")
    subprocess.run([sys.executable, "-m", "deepspeedsyclsupport_amd.launcher.runner", "--num_gpus", "1",
                    "--master_port", "29622", "--autotuning", "tune", str(script), "--deepspeed_config",
                    str(cfg_path)], check=True, env=env, cwd=str(tmp_path), timeout=600)
    summary = json.load(open(tmp_path / "res" / "summary.json"))
    assert summary["best"] is not None and len(summary["records"]) == 4
    assert all(v is not None for _, v in summary["records"])
