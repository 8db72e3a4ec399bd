"""Ragged (FastGen-style) serving engine with the HCache hidden-state cache."""
from .engine import (InferenceEngineV2, RaggedInferenceEngineConfig, SchedulingError, SchedulingResult,  # noqa: F401
                     build_engine_from_ds_checkpoint, build_engine_from_hf_model, build_engine_from_model,
                     build_hf_engine)
from .arch import ArchSpec, convert_hf, spec_from_hf  # noqa: F401
from .ragged import (BlockedAllocator, BlockedKVCache, DSSequenceDescriptor, DSStateManager,  # noqa: F401
                     DSStateManagerConfig, MemoryConfig, RaggedBatchWrapper)
