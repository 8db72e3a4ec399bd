"""Data-efficiency sampling tools: indexed datasets, the offline data analyzer, variable batch size + LR."""
from .data_analyzer import DataAnalyzer, DistributedDataAnalyzer, load_sample_to_metric
from .indexed_dataset import MMapIndexedDataset, MMapIndexedDatasetBuilder, make_builder, make_dataset
from .variable_batch_size_and_lr import (VariableBatchSizeLR, batch_by_seqlens, dataloader_for_variable_batch_size,
                                         get_dataloader_and_lr_scheduler_for_variable_batch_size,
                                         get_dataloader_and_lr_scheduler_for_variable_batch_size_deepspeed,
                                         lr_scheduler_for_variable_batch_size, scale_lr)

__all__ = ["DataAnalyzer", "DistributedDataAnalyzer", "load_sample_to_metric", "MMapIndexedDataset",
           "MMapIndexedDatasetBuilder", "make_builder", "make_dataset", "VariableBatchSizeLR", "batch_by_seqlens",
           "dataloader_for_variable_batch_size", "get_dataloader_and_lr_scheduler_for_variable_batch_size",
           "get_dataloader_and_lr_scheduler_for_variable_batch_size_deepspeed", "lr_scheduler_for_variable_batch_size",
           "scale_lr"]
