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


def _space_metric(exp):
    """Synthetic step throughput: larger buckets help up to 5e8, overlap helps, prefetch 5e8 is the sweet spot."""
    z = exp["ds_config"]["zero_optimization"]
    t = exp["mbs"] * 10.0
    t *= {2e8: 0.9, 5e8: 1.0, 1e9: 0.97}[z.get("reduce_bucket_size", 5e8)]
    t *= 1.05 if z.get("overlap_comm") else 1.0
    t *= {2e8: 0.95, 5e8: 1.0, 1e9: 0.98}.get(z.get("stage3_prefetch_bucket_size", 5e8), 1.0)
    return {"throughput": t}


@pytest.mark.parametrize("tuner", ["gridsearch", "random", "model_based"])
def test_zero_space_tuning_full_mode(tmp_path, tuner):
    base = {"train_micro_batch_size_per_gpu": 1, "zero_optimization": {"stage": 3}, "autotuning": {
        "enabled": True, "fast": False, "tuner_type": tuner, "tuner_early_stopping": 100, "tuner_num_trials": 100,
        "results_dir": str(tmp_path / "res"), "exps_dir": str(tmp_path / "exps"), "zero_stages": [3],
        "max_train_micro_batch_size_per_gpu": 4, "num_tuning_micro_batch_sizes": 1}}
    at = Autotuner(_args([]), {"localhost": list(range(8))}, base_config=base, run_experiment=_space_metric,
                   gpu_mem_bytes=288 * 1024**3, num_params=1e9)
    best = at.tune()
    z = best[0]["ds_config"]["zero_optimization"]
    assert best[0]["mbs"] == 4
    assert z["reduce_bucket_size"] == 5e8 and z["overlap_comm"] is True and z["stage3_prefetch_bucket_size"] == 5e8
    opt = json.load(open(tmp_path / "res" / "ds_config_optimal.json"))
    assert opt["zero_optimization"]["reduce_bucket_size"] == 5e8
    names = [n for n, _ in at.records]
    assert any("reduce_bucket_size" in n for n in names)


def test_model_based_tuner_needs_fewer_trials():
    from deepspeedsyclsupport_amd.autotuning.tuner import GridSearchTuner, ModelBasedTuner
    from deepspeedsyclsupport_amd.autotuning.utils import get_all_configs
    space = {"zero_optimization": {"reduce_bucket_size": [1e8, 2e8, 5e8, 1e9, 2e9], "prefetch": [1e8, 3e8, 1e9, 3e9]}}

    def run(exp):
        z = exp["ds_config"]["zero_optimization"]
        import math
        return {"throughput": -(math.log2(z["reduce_bucket_size"]) - math.log2(5e8))**2 -
                              (math.log2(z["prefetch"]) - math.log2(1e9))**2}

    exps = [{"name": str(i), "ds_config": c} for i, c in enumerate(get_all_configs(space))]
    mb = ModelBasedTuner(list(exps), run, "throughput", space)
    n_mb = mb.tune(sample_size=1, n_trials=20, early_stopping=4)
    assert mb.best_exp["ds_config"]["zero_optimization"] == {"reduce_bucket_size": 5e8, "prefetch": 1e9}
    assert n_mb < len(exps)
    gs = GridSearchTuner(list(exps), run, "throughput")
    gs.tune(sample_size=1, n_trials=100)
    assert gs.best_exp["ds_config"] == mb.best_exp["ds_config"]
