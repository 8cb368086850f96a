"""Tuner loop (reference `tuner/base_tuner.py`): ask for the next batch of experiments, run them through the
resource manager, keep the best by the metric (throughput / FLOPS up, latency down), stop early after
`early_stopping` batches without improvement."""
from ...utils.logging import logger


class BaseTuner:

    def __init__(self, exps, resource_manager, metric):
        self.all_exps = list(exps)
        self.rm = resource_manager
        self.metric = metric
        self.best_exp = None
        self.best_metric_val = None
        self.records = []  # (exp, value or None)

    def has_next(self):
        return len(self.all_exps) > 0

    def next_batch(self, sample_size):
        raise NotImplementedError

    def update(self):
        pass

    def _better(self, v):
        if v is None:
            return False
        if self.best_metric_val is None:
            return True
        return v < self.best_metric_val if self.metric == "latency" else v > self.best_metric_val

    def tune(self, sample_size=1, n_trials=1000, early_stopping=None):
        i, since = 0, 0
        while i < n_trials and self.has_next():
            batch = self.next_batch(sample_size)
            improved = False
            for exp in batch:
                res = self.rm(exp) if callable(self.rm) else self.rm.run_experiment(exp)
                val = None if not res else res.get(self.metric)
                self.records.append((exp, val))
                if self._better(val):
                    self.best_exp, self.best_metric_val, improved = exp, val, True
            self.update()
            i += len(batch)
            since = 0 if improved else since + 1
            if early_stopping is not None and since >= early_stopping:
                logger.info(f"autotuning: early stop after {i} trials ({since} batches without improvement)")
                break
        return i
