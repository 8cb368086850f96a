"""Monitoring backends through the engine (reference `tests/unit/monitor/test_monitor.py`): the CSV monitor writes
the engine's loss / lr events."""
import os

import torch

from ..common import run_distributed
from ..simple_model import base_config, random_tokens, tiny_llama


def _run(logdir):
    import deepspeedsyclsupport_amd as ds
    cfg = base_config(stage=1, lr=1e-3, mb=2, gas=1, clip=1.0)
    cfg["csv_monitor"] = {"enabled": True, "output_path": logdir, "job_name": "job"}
    eng, *_ = ds.initialize(model=tiny_llama(), config=cfg)
    for x in random_tokens(3, 2, 16, seed=1):
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()


def test_csv_monitor(tmp_path):
    run_distributed(_run, 1, str(tmp_path))
    d = tmp_path / "job"
    files = sorted(os.listdir(d))
    assert any("train_loss" in f for f in files) and any("lr" in f for f in files)
    rows = (d / [f for f in files if "train_loss" in f][0]).read_text().strip().splitlines()
    assert len(rows) == 1 + 3 and rows[0].startswith("step")


def test_monitor_config_defaults():
    from deepspeedsyclsupport_amd.runtime.config import DeepSpeedConfig
    c = DeepSpeedConfig({"train_batch_size": 1, "tensorboard": {"enabled": False}})
    assert not c.monitor_config.enabled
