"""``deepspeed.module_inject`` import path (reference module_inject/__init__.py, replace_module.py:183,550,
layers.py:40).

``replace_transformer_layer`` swaps HF BERT-style encoder blocks for the fused training layer
(:class:`~hcache_deepspeed_amd.ops.transformer.DeepSpeedTransformerLayer`, HIP LayerNorm/bias-GELU/attention);
``revert_transformer_layer`` copies the trained weights back into the original block class. Inference-time
kernel injection for decoder LLMs is :func:`hcache_deepspeed_amd.inference.injection.inject`.
"""
import os

import torch
import torch.nn as nn

from ..inference.injection import inject  # noqa: F401
from ..parallel.tp import AutoTP  # noqa: F401


def set_autotp_mode(training=False):
    """Reference layers.py:40: AutoTP linears keep autograd-capable collectives when training."""
    os.environ["DEEPSPEED_AUTOTP_MODE"] = "TRAINING" if training else "INFERENCE"


def _bert_parts(layer):
    att, inter, out = layer.attention, layer.intermediate, layer.output
    return (att.self.query, att.self.key, att.self.value, att.output.dense, att.output.LayerNorm, inter.dense,
            out.dense, out.LayerNorm)


def _ds_config(model_config, config, layer):
    from ..ops.transformer import DeepSpeedTransformerConfig
    q = layer.attention.self.query
    H = q.weight.shape[1]
    heads = getattr(model_config, "num_attention_heads", None) or layer.attention.self.num_attention_heads
    inter = layer.intermediate.dense.weight.shape[0]
    training = bool(getattr(config, "training", True)) if config is not None else True
    return DeepSpeedTransformerConfig(
        batch_size=getattr(config, "train_micro_batch_size_per_gpu", -1) if config is not None else -1,
        hidden_size=H, intermediate_size=inter, heads=heads,
        attn_dropout_ratio=getattr(model_config, "attention_probs_dropout_prob", 0.0),
        hidden_dropout_ratio=getattr(model_config, "hidden_dropout_prob", 0.0),
        num_hidden_layers=getattr(model_config, "num_hidden_layers", 1),
        initializer_range=getattr(model_config, "initializer_range", 0.02),
        layer_norm_eps=getattr(model_config, "layer_norm_eps", 1e-12), pre_layer_norm=False, return_tuple=True,
        training=training)


def replace_transformer_layer(orig_layer_impl, model, checkpoint_dict=None, config=None, model_config=None):
    """Replace every ``orig_layer_impl`` (HF BertLayer-style: post-LN) block of ``model`` with the fused layer,
    copying its weights. Returns the model."""
    from ..ops.transformer import DeepSpeedTransformerLayer
    for parent in list(model.modules()):
        for name, child in list(parent.named_children()):
            if orig_layer_impl is not None and not isinstance(child, orig_layer_impl):
                continue
            if orig_layer_impl is None and not hasattr(child, "attention"):
                continue
            q, k, v, o, ln1, i, out, ln2 = _bert_parts(child)
            new = DeepSpeedTransformerLayer(_ds_config(model_config, config, child)).to(q.weight.device,
                                                                                         q.weight.dtype)
            with torch.no_grad():
                new.attn_qkvw.copy_(torch.cat([q.weight, k.weight, v.weight]))
                new.attn_qkvb.copy_(torch.cat([q.bias, k.bias, v.bias]))
                new.attn_ow.copy_(o.weight)
                new.attn_ob.copy_(o.bias)
                new.attn_nw.copy_(ln1.weight)
                new.attn_nb.copy_(ln1.bias)
                new.inter_w.copy_(i.weight)
                new.inter_b.copy_(i.bias)
                new.output_w.copy_(out.weight)
                new.output_b.copy_(out.bias)
                new.norm_w.copy_(ln2.weight)
                new.norm_b.copy_(ln2.bias)
            new._hds_orig_cls = type(child)
            new._hds_orig_cfg = model_config
            setattr(parent, name, new)
    return model


def revert_transformer_layer(orig_layer_impl, model, config=None, preln=False):
    """Inverse of :func:`replace_transformer_layer`: rebuild ``orig_layer_impl`` blocks with the fused layers'
    (trained) weights."""
    from ..ops.transformer import DeepSpeedTransformerLayer
    for parent in list(model.modules()):
        for name, child in list(parent.named_children()):
            if not isinstance(child, DeepSpeedTransformerLayer):
                continue
            cls = orig_layer_impl or child._hds_orig_cls
            orig = cls(child._hds_orig_cfg if config is None else config)
            q, k, v, o, ln1, i, out, ln2 = _bert_parts(orig)
            H = child.config.hidden_size
            with torch.no_grad():
                qw, kw, vw = child.attn_qkvw.split(H)
                qb, kb, vb = child.attn_qkvb.split(H)
                for lin, w, b in ((q, qw, qb), (k, kw, kb), (v, vw, vb), (o, child.attn_ow, child.attn_ob),
                                  (i, child.inter_w, child.inter_b), (out, child.output_w, child.output_b)):
                    lin.weight.copy_(w)
                    lin.bias.copy_(b)
                for ln, w, b in ((ln1, child.attn_nw, child.attn_nb), (ln2, child.norm_w, child.norm_b)):
                    ln.weight.copy_(w)
                    ln.bias.copy_(b)
            setattr(parent, name, orig.to(child.attn_qkvw.device, child.attn_qkvw.dtype))
    return model


class ReplaceWithTensorSlicing:
    """Reference replace_module.py ReplaceWithTensorSlicing: copy a (TP-sliced) weight into a destination."""

    def __init__(self, mp_group=None, mp_size=1, out_dim=1, in_dim=0):
        self.mp_group, self.mp_size, self.out_dim, self.in_dim = mp_group, mp_size, out_dim, in_dim

    def copy(self, dst, src, int8=False, allocate_tensor=False):
        if src is None:
            return src
        if dst.shape == src.shape:
            dst.data.copy_(src)
            return dst
        rank = torch.distributed.get_rank(self.mp_group) if self.mp_group is not None else 0
        dim = 0 if dst.shape[0] != src.shape[0] else 1
        dst.data.copy_(src.chunk(self.mp_size, dim)[rank])
        return dst


__all__ = ["inject", "AutoTP", "set_autotp_mode", "replace_transformer_layer", "revert_transformer_layer",
           "ReplaceWithTensorSlicing"]
