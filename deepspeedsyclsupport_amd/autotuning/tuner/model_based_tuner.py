"""Model-based tuner (reference `tuner/model_based_tuner.py`): measure a few random points, fit the surrogate
cost model on (features, metric), then always run the untried configuration with the best predicted metric."""
import random

import numpy as np

from ..utils import get_tuning_keys
from .base_tuner import BaseTuner
from .cost_model import RBFCostModel
from .utils import dict_to_feature, flatten

INIT_NUM = 2


class ModelBasedTuner(BaseTuner):

    def __init__(self, exps, resource_manager, metric, tuning_space=None, seed=0):
        super().__init__(exps, resource_manager, metric)
        self.rng = random.Random(seed)
        first = self.all_exps[0]["ds_config"] if self.all_exps else {}
        keys = [k.replace(".", "_") for k in get_tuning_keys(tuning_space)] if tuning_space else None
        self.keys = keys or sorted(flatten(first).keys())
        self.model = RBFCostModel()
        self.trained = False

    def _feat(self, exp):
        return dict_to_feature(exp["ds_config"], self.keys)

    def next_batch(self, sample_size=1):
        measured = [(e, v) for e, v in self.records if v is not None]
        if len(measured) < INIT_NUM or not self.trained:
            k = min(sample_size, len(self.all_exps))
            return [self.all_exps.pop(self.rng.randrange(len(self.all_exps))) for _ in range(k)]
        preds = self.model.predict(np.stack([self._feat(e) for e in self.all_exps]))
        order = np.argsort(preds if self.metric == "latency" else -preds)
        picks = [self.all_exps[i] for i in order[:sample_size]]
        for p in picks:
            self.all_exps.remove(p)
        return picks

    def update(self):
        measured = [(e, v) for e, v in self.records if v is not None]
        if len(measured) >= INIT_NUM:
            self.model.fit(np.stack([self._feat(e) for e, _ in measured]), [v for _, v in measured])
            self.trained = True
