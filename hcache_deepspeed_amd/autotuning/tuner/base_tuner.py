"""Tuner base (reference autotuning/tuner/base_tuner.py ``BaseTuner`` :13): repeatedly pick a batch of experiments,
run them through the experiment runner, keep the best, stop after ``n_trials`` or ``early_stopping`` trials without
improvement."""
from ...utils.logging import logger

METRIC_LATENCY = "latency"


class BaseTuner:

    def __init__(self, exps, runner, metric="throughput"):
        """exps: [{"name": str, "ds_config": dict, ...}]; runner(exp) -> metric dict or None (failed run)."""
        self.all_exps = list(exps)
        self.pending = list(range(len(self.all_exps)))
        self.runner = runner
        self.metric = metric or "throughput"
        self.best_iter = 0
        self.best_exp = None
        self.best_metric_val = None
        self.results = []  # (exp index, metric value or None)

    def _score(self, m):
        if m is None or self.metric not in m:
            return None
        v = float(m[self.metric])
        return -v if self.metric == METRIC_LATENCY else v

    def has_next(self):
        return len(self.pending) > 0

    def next_batch(self, sample_size):
        raise NotImplementedError

    def update(self):
        """Called after every batch with ``self.results`` extended."""

    def tune(self, sample_size=1, n_trials=1000, early_stopping=None):
        i = 0
        while i < n_trials and self.has_next():
            batch = self.next_batch(sample_size)
            if not batch:
                break
            for idx in batch:
                if idx in self.pending:
                    self.pending.remove(idx)
                m = self.runner(self.all_exps[idx])
                score = self._score(m)
                self.results.append((idx, score))
                if score is not None and (self.best_metric_val is None or score > self.best_metric_val):
                    self.best_metric_val, self.best_exp, self.best_iter = score, self.all_exps[idx], i
                i += 1
            self.update()
            if early_stopping and i >= self.best_iter + early_stopping:
                logger.info(f"tuner: early stop at trial {i} (best at {self.best_iter})")
                break
        return i
