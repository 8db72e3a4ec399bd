"""Block-sparse attention (reference deepspeed/ops/sparse_attention): layouts, fused HIP kernel, compressed ops."""
from .bert_sparse_self_attention import BertSparseSelfAttention
from .matmul import MatMul, Softmax
from .sparse_attention_utils import SparseAttentionUtils
from .sparse_self_attention import SparseSelfAttention, block_sparse_attention
from .sparsity_config import (BigBirdSparsityConfig, BSLongformerSparsityConfig, DenseSparsityConfig,
                              FixedSparsityConfig, LocalSlidingWindowSparsityConfig, SparsityConfig,
                              VariableSparsityConfig)

__all__ = [
    "SparsityConfig", "DenseSparsityConfig", "FixedSparsityConfig", "VariableSparsityConfig", "BigBirdSparsityConfig",
    "BSLongformerSparsityConfig", "LocalSlidingWindowSparsityConfig", "SparseSelfAttention", "BertSparseSelfAttention",
    "SparseAttentionUtils", "MatMul", "Softmax", "block_sparse_attention"
]
