"""Difficulty-aware distributed batch sampler (curriculum-by-sample-metric).

Reference parity: runtime/data_pipeline/data_sampling/data_sampler.py (``DeepSpeedDataSampler`` :36): each
global batch is drawn only from samples whose metric value is within the current curriculum difficulty,
the batch is split across data-parallel ranks, and the sampler state (consumed samples, RNG) is
checkpointable. The per-sample metric (e.g. sequence length, vocabulary rarity) comes precomputed as an
array (the reference's data analyzer output), so sampling is a cheap index filter per step.
"""
import numpy as np

from .curriculum_scheduler import CurriculumScheduler


class DeepSpeedDataSampler:

    def __init__(self, metric_values, global_batch_size, micro_batch_size, data_parallel_rank=0,
                 data_parallel_size=1, curriculum_config=None, difficulty_type="value", seed=1234, drop_last=True):
        self.metric = np.asarray(metric_values)
        self.n = len(self.metric)
        self.global_batch_size = int(global_batch_size)
        self.micro_batch_size = int(micro_batch_size)
        self.dp_rank, self.dp_size = int(data_parallel_rank), int(data_parallel_size)
        assert self.global_batch_size % (self.micro_batch_size * self.dp_size) == 0
        self.scheduler = CurriculumScheduler(curriculum_config) if curriculum_config else None
        self.difficulty_type = difficulty_type  # "value" or "percentile"
        self.seed = seed
        self.rng = np.random.default_rng(seed)
        self.consumed_samples = 0
        self.global_step = 0
        self.drop_last = drop_last
        self._order = np.argsort(self.metric, kind="stable")

    @classmethod
    def from_analyzer(cls, save_path, metric_name, global_batch_size, micro_batch_size, **kw):
        """Sampler over the per-sample metric written by the data analyzer (data_sampling/data_analyzer.py; the
        reference's ``<metric>_sample_to_metric`` index files are read the same way)."""
        from .data_sampling.data_analyzer import load_sample_to_metric
        return cls(load_sample_to_metric(save_path, metric_name), global_batch_size, micro_batch_size, **kw)

    def _eligible(self):
        if self.scheduler is None:
            return np.arange(self.n)
        d = self.scheduler.update_difficulty(self.global_step + 1)
        if self.difficulty_type == "percentile":
            k = max(self.global_batch_size, int(self.n * min(100, d) / 100.0))
            return self._order[:k]
        idx = np.nonzero(self.metric <= d)[0]
        if len(idx) < self.global_batch_size:  # not enough easy samples yet: take the easiest ones
            idx = self._order[:self.global_batch_size]
        return idx

    def get_next_global_batch(self):
        idx = self._eligible()
        batch = self.rng.choice(idx, size=self.global_batch_size, replace=len(idx) < self.global_batch_size)
        self.consumed_samples += self.global_batch_size
        self.global_step += 1
        return batch

    def __iter__(self):
        while True:
            batch = self.get_next_global_batch()
            per_rank = self.global_batch_size // self.dp_size
            mine = batch[self.dp_rank * per_rank:(self.dp_rank + 1) * per_rank]
            for i in range(0, per_rank, self.micro_batch_size):
                yield mine[i:i + self.micro_batch_size].tolist()

    def __len__(self):
        return self.n // self.global_batch_size

    def state_dict(self):
        return {"consumed_samples": self.consumed_samples, "global_step": self.global_step,
                "rng": self.rng.bit_generator.state,
                "curriculum": self.scheduler.get_state() if self.scheduler else None}

    def load_state_dict(self, sd):
        self.consumed_samples = sd["consumed_samples"]
        self.global_step = sd["global_step"]
        self.rng.bit_generator.state = sd["rng"]
        if self.scheduler is not None and sd.get("curriculum"):
            self.scheduler.set_state(sd["curriculum"])
