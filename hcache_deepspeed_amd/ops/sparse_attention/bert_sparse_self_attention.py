"""BERT self-attention with block-sparse attention (reference ops/sparse_attention/bert_sparse_self_attention.py)."""
import torch.nn as nn

from .sparse_self_attention import SparseSelfAttention
from .sparsity_config import FixedSparsityConfig


class BertSparseSelfAttention(nn.Module):
    """Drop-in for HF ``BertSelfAttention``: Q/K/V projections + :class:`SparseSelfAttention`.

    ``config`` needs ``hidden_size`` and ``num_attention_heads``; forward(hidden_states [B, S, H],
    attention_mask [B, S] additive key-padding mask) -> context [B, S, H].
    """

    def __init__(self, config, sparsity_config=None):
        super().__init__()
        if config.hidden_size % config.num_attention_heads != 0:
            raise ValueError(f"The hidden size ({config.hidden_size}) is not a multiple of the number of attention "
                             f"heads ({config.num_attention_heads})")
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = config.hidden_size // config.num_attention_heads
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        if sparsity_config is None:
            sparsity_config = FixedSparsityConfig(num_heads=config.num_attention_heads)
        self.sparse_self_attention = SparseSelfAttention(sparsity_config)

    def transpose_for_scores(self, x):
        new_x_shape = x.size()[:-1] + (self.num_attention_heads, self.attention_head_size)
        return x.view(*new_x_shape).permute(0, 2, 1, 3)

    def forward(self, hidden_states, attention_mask=None):
        q = self.transpose_for_scores(self.query(hidden_states))
        k = self.transpose_for_scores(self.key(hidden_states))
        v = self.transpose_for_scores(self.value(hidden_states))
        ctx = self.sparse_self_attention(q, k, v, key_padding_mask=attention_mask)
        ctx = ctx.permute(0, 2, 1, 3).contiguous()
        return ctx.view(*ctx.size()[:-2], self.all_head_size)
