"""bench.py driver contract on the CPU: the multi-rank launch (`torch.distributed.run --nproc-per-node N bench.py
--gpus N`) must run the DP / Ulysses-SP control flow and print exactly ONE JSON line from rank 0 with the keys
the driver reads. `--host-dryrun` swaps in gloo and a tiny Llama (a plumbing check, not a measurement)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("extra", [[], ["--sp", "2"], ["--zero-init", "--offload-ratio", "0.5"]],
                         ids=["dp2", "sp2", "zeroinit-twinflow"])
def test_bench_two_rank_dryrun_prints_one_json_line(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--host-dryrun"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec), sorted(KEYS - set(rec))
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True
    assert rec["config"]["parallelism"] == ("dp1-sp2" if "--sp" in extra else "dp2")
    assert rec["final_loss"] == rec["final_loss"]  # not NaN


def test_top_level_api_names():
    """Every public top-level name of the reference's `deepspeed/__init__.py` resolves here."""
    import deepspeedsyclsupport_amd as ds
    for name in ("initialize", "init_inference", "init_distributed", "add_config_arguments", "default_inference_config",
                 "DeepSpeedEngine", "DeepSpeedHybridEngine", "PipelineEngine", "PipelineModule", "InferenceEngine",
                 "DeepSpeedInferenceConfig", "DeepSpeedConfig", "DeepSpeedConfigError", "checkpointing",
                 "DeepSpeedTransformerLayer", "DeepSpeedTransformerConfig", "replace_transformer_layer",
                 "revert_transformer_layer", "OnDevice", "zero", "DeepSpeedOptimizer", "ZeROOptimizer",
                 "ADAM_OPTIMIZER", "LAMB_OPTIMIZER", "log_dist", "logger", "get_accelerator", "add_tuning_arguments",
                 "ops", "module_inject", "comm", "version", "git_hash", "git_branch"):
        assert getattr(ds, name) is not None or name in ("git_hash", "git_branch"), name
