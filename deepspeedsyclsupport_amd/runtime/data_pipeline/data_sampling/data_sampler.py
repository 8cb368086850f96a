"""Curriculum data sampler (reference `runtime/data_pipeline/data_sampling/data_sampler.py`).

Each sample has a difficulty metric value (e.g. sequence length or vocabulary rarity, precomputed by an analyzer
and stored as a numpy array / memmap). At every step the sampler draws the global batch only from samples whose
metric is <= the scheduler's current difficulty (`value` clustering) or from the easiest `difficulty` percentile
(`percentile`), shuffled with a seed shared by all ranks, and hands each data-parallel rank its slice.
"""
import numpy as np

from ..curriculum_scheduler import CurriculumScheduler


def _values_from_index(index_to_sample_path, index_to_metric_path, total):
    """Per-sample difficulty from the analyzer's value-grouped index (group ordinal if no metric file is given)."""
    from .indexed_dataset import MMapIndexedDataset
    i2s = MMapIndexedDataset(index_to_sample_path)
    i2m = MMapIndexedDataset(index_to_metric_path) if index_to_metric_path else None
    vals = np.zeros(total, dtype=np.int64)
    for row in range(len(i2s)):
        vals[np.asarray(i2s[row], dtype=np.int64)] = int(i2m[row][0]) if i2m is not None else row
    return vals


def _load_sample_to_metric(path):
    """A .npy array (loaded without pickle) or an MMIDIDX `<prefix>_sample_to_metric` dataset."""
    if path.endswith(".npy"):
        return np.load(path, mmap_mode="r")
    from .indexed_dataset import MMapIndexedDataset
    ds = MMapIndexedDataset(path)
    return np.concatenate(ds[0:len(ds)]).astype(np.int64)


class DeepSpeedDataSampler:

    def __init__(self, data_efficiency_config, one_epoch_total_samples, micro_batch_size, data_parallel_rank,
                 data_parallel_size, gradient_accumulation_steps=1, global_rank=0, drop_last=True,
                 metric_values=None):
        self.cfg = data_efficiency_config
        cl = self.cfg.get("data_sampling", {}).get("curriculum_learning", {})
        self.total = int(one_epoch_total_samples)
        self.mb = micro_batch_size
        self.dp_rank, self.dp_size = data_parallel_rank, data_parallel_size
        self.gas = gradient_accumulation_steps
        self.global_batch = micro_batch_size * data_parallel_size * gradient_accumulation_steps
        self.seed = int(self.cfg.get("seed", 1234))
        self.metrics = {}
        self.schedulers = {}
        for name, mc in cl.get("curriculum_metrics", {}).items():
            self.schedulers[name] = CurriculumScheduler(mc)
            vals = metric_values.get(name) if metric_values else None
            if vals is None and mc.get("index_to_sample_path"):
                # DataAnalyzer output (reference config keys index_to_sample_path / index_to_metric_path)
                vals = _values_from_index(mc["index_to_sample_path"], mc.get("index_to_metric_path"), self.total)
            if vals is None and mc.get("sample_to_metric_path"):
                vals = _load_sample_to_metric(mc["sample_to_metric_path"])
            self.metrics[name] = (np.asarray(vals), mc.get("difficulty_type", "value"))
        self.consumed_samples = 0
        self.curriculum_step = 0
        self.np_rng = np.random.default_rng(self.seed)

    def __len__(self):
        return self.total

    def set_custom_curriculum_learning_schedule(self, schedule_func_dict):
        """{metric name: fn(global step) -> difficulty} for metrics whose schedule_type is "custom" (reference
        `data_sampling/data_sampler.py:97-100`)."""
        for name, fn in schedule_func_dict.items():
            if name in self.schedulers:
                self.schedulers[name].set_custom_get_difficulty(fn)

    def _eligible(self):
        mask = np.ones(self.total, dtype=bool)
        for name, (vals, dtype) in self.metrics.items():
            d = self.schedulers[name].update_difficulty(self.curriculum_step)
            if dtype == "percentile":
                thr = np.percentile(vals, d)
                mask &= vals <= thr
            else:
                mask &= vals <= d
        idx = np.nonzero(mask)[0]
        return idx if idx.size else np.arange(self.total)

    def get_next_global_batch(self):
        self.curriculum_step += 1
        pool = self._eligible()
        batch = self.np_rng.choice(pool, size=self.global_batch, replace=pool.size < self.global_batch)
        self.consumed_samples += self.global_batch
        return batch

    def __iter__(self):
        while self.consumed_samples < self.total:
            gb = self.get_next_global_batch()
            per_rank = gb.reshape(self.gas, self.dp_size, self.mb)[:, self.dp_rank]
            for micro in per_rank:
                yield micro.tolist()

    def state_dict(self):
        return {"consumed_samples": self.consumed_samples, "curriculum_step": self.curriculum_step,
                "rng": self.np_rng.bit_generator.state,
                "schedulers": {k: s.get_state() for k, s in self.schedulers.items()}}

    def load_state_dict(self, sd):
        self.consumed_samples = sd["consumed_samples"]
        self.curriculum_step = sd["curriculum_step"]
        self.np_rng.bit_generator.state = sd["rng"]
        for k, st in sd["schedulers"].items():
            self.schedulers[k].set_state(st)
