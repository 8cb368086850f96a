"""Grid-search and random tuners (reference `tuner/index_based_tuner.py`)."""
import random

from .base_tuner import BaseTuner


class GridSearchTuner(BaseTuner):

    def next_batch(self, sample_size=1):
        batch, self.all_exps = self.all_exps[:sample_size], self.all_exps[sample_size:]
        return batch


class RandomTuner(BaseTuner):

    def __init__(self, exps, resource_manager, metric, seed=0):
        super().__init__(exps, resource_manager, metric)
        self.rng = random.Random(seed)

    def next_batch(self, sample_size=1):
        batch = []
        for _ in range(min(sample_size, len(self.all_exps))):
            batch.append(self.all_exps.pop(self.rng.randrange(len(self.all_exps))))
        return batch
