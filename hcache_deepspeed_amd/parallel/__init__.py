"""Parallelism strategies: tensor (AutoTP), sequence (Ulysses, FPDT), expert (MoE)."""
from .fpdt import (FPDT_Attention, FPDT_FFN, FPDT_LogitsLoss, FPDTInputConstruct, chunked_apply,  # noqa: F401
                   enable_fpdt, fpdt_attention)
from .ulysses import DistributedAttention, enable_sequence_parallel  # noqa: F401
