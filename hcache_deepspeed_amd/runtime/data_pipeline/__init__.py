"""Data efficiency: curriculum learning scheduler, difficulty-aware sampler, random layerwise token dropping."""
from .curriculum_scheduler import CurriculumScheduler
from .data_sampler import DeepSpeedDataSampler
from .data_sampling import (DataAnalyzer, DistributedDataAnalyzer, MMapIndexedDataset, MMapIndexedDatasetBuilder,
                            VariableBatchSizeLR, batch_by_seqlens,
                            get_dataloader_and_lr_scheduler_for_variable_batch_size, scale_lr)
from .random_ltd import RandomLayerTokenDrop, RandomLTDScheduler, gpt_sample_tokens, token_gather, token_scatter

__all__ = ["CurriculumScheduler", "DeepSpeedDataSampler", "DataAnalyzer", "DistributedDataAnalyzer",
           "MMapIndexedDataset", "MMapIndexedDatasetBuilder", "VariableBatchSizeLR", "batch_by_seqlens",
           "get_dataloader_and_lr_scheduler_for_variable_batch_size", "scale_lr", "RandomLayerTokenDrop", "RandomLTDScheduler",
           "gpt_sample_tokens", "token_gather", "token_scatter"]
