"""Model compression library (QAT, pruning, layer reduction) -- reference deepspeed/compression."""
from .compress import (compression_scheduler, fix_compression, get_compress_methods, get_module_name,
                       init_compression, module_replacement, recursive_getattr, recursive_setattr, redundancy_clean,
                       student_initialization)
from .config import get_compression_config
from .layers import (BNLayer_Compress, ColumnParallelLinear_Compress, Conv2dLayer_Compress, Embedding_Compress,
                     LinearLayer_Compress, QuantAct, RowParallelLinear_Compress, TopKBinarizer)

__all__ = [
    "init_compression", "redundancy_clean", "student_initialization", "compression_scheduler",
    "get_compression_config", "LinearLayer_Compress", "Conv2dLayer_Compress", "Embedding_Compress",
    "BNLayer_Compress", "ColumnParallelLinear_Compress", "RowParallelLinear_Compress", "TopKBinarizer", "QuantAct",
    "fix_compression", "module_replacement", "get_module_name", "get_compress_methods", "recursive_getattr",
    "recursive_setattr"
]
