"""Model-based tuner (reference autotuning/tuner/model_based_tuner.py ``ModelBasedTuner`` :19): a few initial
trials, then a cost model fitted on the measured configurations ranks the untried ones; each batch takes the top
predictions, with a fraction of random picks to keep exploring."""
import numpy as np

from .base_tuner import BaseTuner
from .cost_model import CostModel
from .utils import dict_to_feature, flatten

INIT_NUM = 2


class ModelBasedTuner(BaseTuner):

    def __init__(self, exps, runner, metric="throughput", tuning_space=None, seed=0, random_exploration_ratio=0.2):
        super().__init__(exps, runner, metric)
        self.tuning_space = tuning_space or {}
        self.rng = np.random.default_rng(seed)
        flat = [flatten(e["ds_config"]) for e in self.all_exps]
        keys = sorted({k for f in flat for k, v in f.items() if isinstance(v, (int, float, bool))})
        # keep only the keys that actually vary: constant features carry no signal
        keys = [k for k in keys if len({f.get(k) for f in flat}) > 1]
        mx = {k: max(abs(float(f.get(k, 0) or 0)) for f in flat) or 1.0 for k in keys}
        self.features = np.array([dict_to_feature(f, keys, mx) for f in flat], dtype=np.float64)
        self.cost_model = CostModel("rank", seed=seed)
        self.random_exploration_ratio = random_exploration_ratio
        n0 = min(INIT_NUM, len(self.all_exps))
        self.init_trials = list(self.rng.choice(len(self.all_exps), size=n0, replace=False)) if n0 else []

    def next_batch(self, sample_size=1):
        out = []
        while len(out) < sample_size and self.pending:
            avail = [i for i in self.pending if i not in out]
            if not avail:
                break
            first = [i for i in self.init_trials if i in avail]
            measured = [(i, s) for i, s in self.results if s is not None]
            if first:
                out.append(first[0])
            elif len(measured) < 2 or self.rng.random() < self.random_exploration_ratio:
                out.append(int(self.rng.choice(avail)))
            else:
                pred = self.cost_model.predict(self.features[avail])
                out.append(avail[int(np.argmax(pred))])
        return out

    def update(self):
        measured = [(i, s) for i, s in self.results if s is not None]
        if len(measured) >= 2:
            xs = self.features[[i for i, _ in measured]]
            ys = [s for _, s in measured]
            self.cost_model.fit(xs, ys)
