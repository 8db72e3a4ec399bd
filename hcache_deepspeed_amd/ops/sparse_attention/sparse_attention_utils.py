"""Helpers to retrofit block-sparse attention into pretrained BERT / RoBERTa models.

Reference parity: ops/sparse_attention/sparse_attention_utils.py (``SparseAttentionUtils``:
``extend_position_embedding``, ``update_tokenizer_model_max_length``,
``replace_model_self_attention_with_sparse_self_attention``,
``replace_self_attention_layer_with_sparse_self_attention_layer``, ``pad_to_block_size``,
``unpad_sequence_output``).
"""
import torch
import torch.nn.functional as F

from .bert_sparse_self_attention import BertSparseSelfAttention
from .sparsity_config import SparsityConfig


class SparseAttentionUtils:

    @staticmethod
    def extend_position_embedding(model, max_position):
        """Tile the learned position embeddings up to ``max_position`` (RoBERTa keeps its 2 reserved rows)."""
        if hasattr(model, "bert"):
            emb = model.bert.embeddings.position_embeddings
            orig = emb.weight.size(0)
            assert max_position > orig
            reps = max(1, max_position // orig)
            emb.weight.data = emb.weight.data.repeat(reps, 1)
            emb.num_embeddings = emb.weight.shape[0]
        elif hasattr(model, "roberta"):
            emb = model.roberta.embeddings.position_embeddings
            orig, dim = emb.weight.shape
            orig -= 2
            assert max_position > orig
            reps = max(1, max_position // orig)
            new = emb.weight.data.new_empty(orig * reps + 2, dim)
            new[:2] = emb.weight.data[:2]
            for i in range(reps):
                new[2 + i * orig:2 + (i + 1) * orig] = emb.weight.data[2:]
            emb.weight.data = new
            emb.num_embeddings = new.shape[0]
            max_position += 2
        else:
            raise ValueError("extend_position_embedding supports models with a 'bert' or 'roberta' attribute")
        model.config.max_position_embeddings = max_position
        return model

    @staticmethod
    def update_tokenizer_model_max_length(tokenizer, max_position):
        tokenizer.model_max_length = max_position
        tokenizer.init_kwargs["model_max_length"] = max_position
        return tokenizer

    @staticmethod
    def replace_model_self_attention_with_sparse_self_attention(model, max_position,
                                                                sparsity_config=SparsityConfig(num_heads=4)):
        if hasattr(model, "bert"):
            model.config.max_position_embeddings = max_position
            layers = model.bert.encoder.layer
        elif hasattr(model, "roberta"):
            model.config.max_position_embeddings = max_position + 2
            layers = model.roberta.encoder.layer
        else:
            raise ValueError("replace_model_self_attention_with_sparse_self_attention supports 'bert' or 'roberta'")
        SparseAttentionUtils.replace_self_attention_layer_with_sparse_self_attention_layer(
            model.config, layers, sparsity_config)
        return model

    @staticmethod
    def replace_self_attention_layer_with_sparse_self_attention_layer(config, layers,
                                                                      sparsity_config=SparsityConfig(num_heads=4)):
        for layer in layers:
            old = layer.attention.self
            new = BertSparseSelfAttention(config, sparsity_config)
            new.query, new.key, new.value = old.query, old.key, old.value
            layer.attention.self = new
        return layers

    @staticmethod
    def pad_to_block_size(block_size, input_ids, attention_mask, token_type_ids, position_ids, inputs_embeds,
                          pad_token_id, model_embeddings):
        """Right-pad every sequence input to a multiple of ``block_size``; returns (pad_len, *padded inputs)."""
        batch_size, seq_len = input_ids.shape[:2] if input_ids is not None else inputs_embeds.shape[:2]
        pad_len = (block_size - seq_len % block_size) % block_size
        if pad_len > 0:
            if inputs_embeds is not None:
                pad_ids = inputs_embeds.new_full((batch_size, pad_len), pad_token_id, dtype=torch.long)
                inputs_embeds = torch.cat([inputs_embeds, model_embeddings(pad_ids)], dim=-2)
            if input_ids is not None:
                input_ids = F.pad(input_ids, (0, pad_len), value=pad_token_id)
            if position_ids is not None:
                position_ids = F.pad(position_ids, (0, pad_len), value=pad_token_id)
            attention_mask = F.pad(attention_mask, (0, pad_len), value=False)
            token_type_ids = F.pad(token_type_ids, (0, pad_len), value=0)
        return pad_len, input_ids, attention_mask, token_type_ids, position_ids, inputs_embeds

    @staticmethod
    def unpad_sequence_output(pad_len, sequence_output):
        if pad_len > 0:
            sequence_output = sequence_output[:, :-pad_len]
        return sequence_output
