"""ZeRO / micro-batch autotuner (reference `autotuning/autotuner.py:42-1100`, `scheduler.py:33`, `tuner/*`).

Flow (same contract as the reference):
  1. model info: one short profiling run reports the parameter count (engine writes `model_info.json` when
     `autotuning.model_info.profile` is set);
  2. per ZeRO stage, a memory model (bytes/param of weights, grads, optimizer states under that stage's
     partitioning, plus activation headroom) prunes stages that cannot fit the per-GPU HBM (288 GB on MI355X);
  3. for the surviving stages, candidate micro-batch sizes (powers of two between the min and the largest that the
     memory model admits, at most `num_tuning_micro_batch_sizes` per stage) are run as experiments — each is the
     user script launched with a derived DeepSpeed config whose engine measures `metric` between
     start_profile_step and end_profile_step and writes it to `metric_path`, then exits;
  4. gridsearch / random / model-based (fit metric ~ mbs per stage, try the predicted best first) ordering with
     early stopping;
  5. unless `autotuning.fast` (default true), the ZeRO knobs of the winning stage are tuned at its micro-batch size
     over a tuning space (`autotuning.tuning_space` or `config_templates.DEFAULT_TUNING_SPACE`: bucket sizes,
     overlap, stage-3 prefetch / live-parameter / persistence budgets) with the `tuner/` grid, random or
     model-based (surrogate cost model) tuner; the best config is written to `results_dir/ds_config_optimal.json`.
Experiments are launched through `launcher.runner` (or a caller-supplied `run_experiment` callable, used in tests).
"""
import copy
import itertools
import json
import math
import os
import random
import subprocess
import sys

from ..utils.logging import logger
from .config_templates import DEFAULT_TUNING_SPACE
from .tuner import GridSearchTuner, ModelBasedTuner, RandomTuner
from .utils import canonical_name, get_all_configs, get_tuning_keys, merge

GB = 1024**3


class ResourceManager:
    """Runs experiments one after another on the given hosts (reference `scheduler.py:33`)."""

    def __init__(self, args, hosts, num_gpus_per_node, results_dir, exps_dir, arg_mappings=None):
        self.args = args
        self.hosts = hosts
        self.num_gpus_per_node = num_gpus_per_node
        self.results_dir = results_dir
        self.exps_dir = exps_dir
        self.arg_mappings = arg_mappings or {}

    def run_experiment(self, exp):
        exp_dir = os.path.join(self.exps_dir, exp["name"])
        os.makedirs(exp_dir, exist_ok=True)
        cfg_path = os.path.join(exp_dir, "ds_config.json")
        with open(cfg_path, "w") as f:
            json.dump(exp["ds_config"], f)
        user_args = list(self.args.user_args)
        if "--deepspeed_config" in user_args:
            user_args[user_args.index("--deepspeed_config") + 1] = cfg_path
        else:
            user_args += ["--deepspeed_config", cfg_path]
        for ds_key, arg_name in self.arg_mappings.items():
            val = exp["ds_config"].get(ds_key)
            if val is not None:
                if arg_name in user_args:
                    user_args[user_args.index(arg_name) + 1] = str(val)
                else:
                    user_args += [arg_name, str(val)]
        cmd = [sys.executable, "-m", "deepspeedsyclsupport_amd.launcher.runner", "--num_gpus",
               str(self.num_gpus_per_node), self.args.user_script] + user_args
        with open(os.path.join(exp_dir, "stdout.log"), "w") as out:
            rc = subprocess.run(cmd, stdout=out, stderr=subprocess.STDOUT).returncode
        return _read_metric(exp["ds_config"]["autotuning"]["metric_path"]) if rc == 0 else None


def _read_metric(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


class Autotuner:

    def __init__(self, args, active_resources, base_config=None, run_experiment=None, gpu_mem_bytes=None,
                 num_params=None):
        self.args = args
        self.resources = active_resources
        if base_config is None:
            path = _find_config_arg(args.user_args)
            with open(path) as f:
                base_config = json.load(f)
        self.base = base_config
        at = base_config.get("autotuning", {})
        from .config import DeepSpeedAutotuningConfig
        DeepSpeedAutotuningConfig(**at)  # unknown keys / wrong types fail here, before any experiment is launched
        self.at = at
        self.results_dir = at.get("results_dir", "autotuning_results")
        self.exps_dir = at.get("exps_dir", "autotuning_exps")
        os.makedirs(self.results_dir, exist_ok=True)
        os.makedirs(self.exps_dir, exist_ok=True)
        self.metric = at.get("metric", "throughput")
        self.tuner_type = at.get("tuner_type", "gridsearch")
        self.early_stop = at.get("tuner_early_stopping", 5)
        self.num_trials = at.get("tuner_num_trials", 50)
        self.min_mbs = at.get("min_train_micro_batch_size_per_gpu", 1)
        self.max_mbs = at.get("max_train_micro_batch_size_per_gpu", 1024)
        self.num_mbs = at.get("num_tuning_micro_batch_sizes", 3)
        self.mp_size = at.get("mp_size", 1)
        self.n_gpus = sum(len(v) for v in active_resources.values()) if active_resources else 1
        self.gpu_mem = gpu_mem_bytes or _device_mem()
        self.num_params = num_params
        self.activation_bytes_per_sample = at.get("activation_mem_per_sample", None)
        self.rm = None if run_experiment is not None else ResourceManager(
            args, list(active_resources), max(len(v) for v in active_resources.values()), self.results_dir,
            self.exps_dir, at.get("arg_mappings"))
        self._run = run_experiment or self.rm.run_experiment
        self.records = []

    # ------------------------------------------------------------------------------------------ memory model
    def model_state_bytes(self, stage, n_params=None):
        """Per-GPU bytes of weights + grads + Adam states (bf16/fp16 weights & grads, fp32 master + 2 moments)."""
        n = n_params or self.num_params
        dp = max(self.n_gpus // self.mp_size, 1)
        n = n / self.mp_size
        w, g, opt = 2 * n, 2 * n, 12 * n
        if stage >= 1:
            opt /= dp
        if stage >= 2:
            g /= dp
        if stage >= 3:
            w /= dp
        return w + g + opt

    def max_mbs_for(self, stage):
        free = 0.9 * self.gpu_mem - self.model_state_bytes(stage)
        if free <= 0:
            return 0
        if not self.activation_bytes_per_sample:
            return self.max_mbs
        return int(min(self.max_mbs, free // self.activation_bytes_per_sample))

    # ------------------------------------------------------------------------------------------ experiments
    def _exp(self, stage, mbs):
        cfg = copy.deepcopy(self.base)
        cfg.setdefault("zero_optimization", {})["stage"] = stage
        cfg["train_micro_batch_size_per_gpu"] = mbs
        cfg.pop("train_batch_size", None)
        gas = cfg.get("gradient_accumulation_steps", 1)
        cfg["gradient_accumulation_steps"] = gas
        name = f"z{stage}_mbs{mbs}"
        at = dict(self.at)
        at.update(enabled=True, metric_path=os.path.join(self.exps_dir, name, "metrics.json"))
        cfg["autotuning"] = at
        return {"name": name, "ds_config": cfg, "stage": stage, "mbs": mbs}

    def _candidates(self, stage):
        hi = self.max_mbs_for(stage)
        if hi < self.min_mbs:
            return []
        vals = sorted({min(hi, 2**k) for k in range(int(math.log2(max(self.min_mbs, 1))), int(math.log2(hi)) + 1)}
                      | {hi})
        vals = [v for v in vals if v >= self.min_mbs]
        return vals[-self.num_mbs:] if len(vals) > self.num_mbs else vals

    def _order(self, exps):
        if self.tuner_type == "random":
            random.Random(0).shuffle(exps)
        elif self.tuner_type == "model_based":
            exps.sort(key=lambda e: -e["mbs"])  # throughput grows with mbs until memory runs out: largest first
        return exps

    def tune(self):
        stages = self.at.get("zero_stages", [0, 1, 2, 3])
        if self.num_params is None:
            self.num_params = self.profile_model_info()
        exps = []
        for st in stages:
            if self.max_mbs_for(st) < self.min_mbs:
                logger.info(f"autotuning: ZeRO-{st} does not fit ({self.model_state_bytes(st) / GB:.1f} GB states)")
                continue
            exps += [self._exp(st, m) for m in self._candidates(st)]
        exps = self._order(exps)[:self.num_trials]
        best, since = None, 0
        for e in exps:
            res = self._run(e)
            val = None if not res else res.get(self.metric)
            self.records.append((e["name"], val))
            if self._better(val, best):
                best, since = (e, val), 0
            else:
                since += 1
                if since >= self.early_stop:
                    break
        if best is not None and not self.at.get("fast", True):
            tuned = self.tune_space(best[0]["stage"], best[0]["mbs"])
            if tuned is not None and self._better(tuned[1], best):
                best = tuned
        self.best = best
        if best is not None:
            out = copy.deepcopy(best[0]["ds_config"])
            out.pop("autotuning", None)
            with open(os.path.join(self.results_dir, "ds_config_optimal.json"), "w") as f:
                json.dump(out, f, indent=2)
        with open(os.path.join(self.results_dir, "summary.json"), "w") as f:
            json.dump({"records": self.records, "best": best[0]["name"] if best else None,
                       "metric": self.metric, "best_value": best[1] if best else None}, f, indent=2)
        return best

    def _better(self, val, best):
        return val is not None and (best is None or (val < best[1] if self.metric == "latency" else val > best[1]))

    def tune_space(self, stage, mbs):
        """Tune the ZeRO knobs of `stage` at micro-batch `mbs` over the tuning space (step 5 above)."""
        space = copy.deepcopy(self.at.get("tuning_space") or DEFAULT_TUNING_SPACE.get(stage, {}))
        space.setdefault("zero_optimization", {})["stage"] = stage
        keys = get_tuning_keys(space)
        exps = []
        for point in get_all_configs(space):
            cfg = merge(self.base, point)
            cfg["train_micro_batch_size_per_gpu"] = mbs
            cfg.pop("train_batch_size", None)
            name = canonical_name(cfg, keys)
            at = dict(self.at)
            at.update(enabled=True, metric_path=os.path.join(self.exps_dir, name, "metrics.json"))
            cfg["autotuning"] = at
            exps.append({"name": name, "ds_config": cfg, "stage": stage, "mbs": mbs})
        if len(exps) <= 1:
            return None
        if self.tuner_type == "model_based":
            tuner = ModelBasedTuner(exps, self._run, self.metric, space)
        elif self.tuner_type == "random":
            tuner = RandomTuner(exps, self._run, self.metric)
        else:
            tuner = GridSearchTuner(exps, self._run, self.metric)
        tuner.tune(sample_size=1, n_trials=self.num_trials, early_stopping=self.early_stop)
        self.records += [(e["name"], v) for e, v in tuner.records]
        return (tuner.best_exp, tuner.best_metric_val) if tuner.best_exp is not None else None

    def profile_model_info(self):
        exp = self._exp(0, self.min_mbs)
        exp["name"] = "profile_model_info"
        info_path = os.path.join(self.exps_dir, "profile_model_info", "model_info.json")
        exp["ds_config"]["autotuning"].update(model_info={"profile": True}, model_info_path=info_path)
        res = self._run(exp)
        if res and "num_params" in res:
            return res["num_params"]
        info = _read_metric(info_path)
        if not info:
            raise RuntimeError("autotuning: model info profiling run failed")
        return info["num_params"]

    def print_tuning_results(self):
        for name, val in self.records:
            logger.info(f"{name}: {self.metric}={val}")
        if getattr(self, "best", None):
            logger.info(f"best: {self.best[0]['name']} {self.metric}={self.best[1]}")


def _find_config_arg(user_args):
    for flag in ("--deepspeed_config", "--deepspeed-config"):
        if flag in user_args:
            return user_args[user_args.index(flag) + 1]
    raise ValueError("autotuning needs --deepspeed_config <path> in the user script arguments")


def _device_mem():
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.get_device_properties(0).total_memory
    except Exception:
        pass
    return 288 * GB
