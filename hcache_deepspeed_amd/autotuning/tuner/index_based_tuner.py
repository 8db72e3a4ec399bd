"""Index-based tuners (reference autotuning/tuner/index_based_tuner.py): grid order and uniform random order."""
import random

from .base_tuner import BaseTuner


class GridSearchTuner(BaseTuner):

    def next_batch(self, sample_size=1):
        return self.pending[:sample_size]


class RandomTuner(BaseTuner):

    def __init__(self, exps, runner, metric="throughput", seed=None):
        super().__init__(exps, runner, metric)
        self.rng = random.Random(seed)

    def next_batch(self, sample_size=1):
        k = min(sample_size, len(self.pending))
        return self.rng.sample(self.pending, k)
