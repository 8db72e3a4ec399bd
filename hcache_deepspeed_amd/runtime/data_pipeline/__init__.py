"""Data efficiency: curriculum learning scheduler, difficulty-aware sampler, random layerwise token dropping."""
from .curriculum_scheduler import CurriculumScheduler
from .data_sampler import DeepSpeedDataSampler
from .random_ltd import RandomLayerTokenDrop, RandomLTDScheduler, gpt_sample_tokens, token_gather, token_scatter

__all__ = ["CurriculumScheduler", "DeepSpeedDataSampler", "RandomLayerTokenDrop", "RandomLTDScheduler",
           "gpt_sample_tokens", "token_gather", "token_scatter"]
