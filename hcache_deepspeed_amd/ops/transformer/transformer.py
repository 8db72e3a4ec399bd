"""Fused BERT-style transformer layer for training (pre- or post-LayerNorm encoder block).

Reference parity: ops/transformer/transformer.py (``DeepSpeedTransformerConfig`` :34, ``DeepSpeedTransformerLayer``
:296 with parameters attn_qkvw/attn_qkvb/attn_ow/attn_ob/attn_nw/attn_nb/inter_w/inter_b/output_w/output_b/
norm_w/norm_b; forward(hidden_states, attention_mask) ) backed by csrc/transformer/*.cu (6.6k LoC: cuBLAS GEMMs,
fused bias+residual LayerNorm, softmax, bias+GeLU, dropout, 0213 transforms).

MI355X composition of the same layer from this framework's HIP kernels instead of a monolithic C++ layer object:
fused residual-add + LayerNorm (norm.hip, fwd/bwd), fused bias + GeLU (act.hip), FlashAttention (flash_attn.hip,
non-causal, head_dim 128, no score matrix) and hipBLASLt GEMMs for the four projections. When an additive
attention mask, attention dropout or another head size is present the attention runs as fp32-softmax torch
math with the same semantics. ``normalize_invertible`` / ``gelu_checkpoint`` / ``attn_dropout_checkpoint`` are
memory knobs of the CUDA layer; here the equivalent saving comes from the fused kernels not keeping
intermediates (they are accepted and recorded).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..activations import bias_act
from ..attention import flash_attn, native_supported, padding_mask_lengths
from ..norm import layer_norm


class TransformerConfig:

    def __init__(self, batch_size, hidden_size, intermediate_size, heads, attn_dropout_ratio, hidden_dropout_ratio,
                 num_hidden_layers, initializer_range):
        self.layer_id = -1
        self.batch_size = batch_size
        self.hidden_size = hidden_size
        self.intermediate_size = intermediate_size
        self.heads = heads
        self.attn_dropout_ratio = attn_dropout_ratio
        self.hidden_dropout_ratio = hidden_dropout_ratio
        self.num_hidden_layers = num_hidden_layers
        self.initializer_range = initializer_range


class DeepSpeedTransformerConfig(TransformerConfig):

    def __init__(self, batch_size=-1, hidden_size=-1, intermediate_size=-1, heads=-1, attn_dropout_ratio=-1,
                 hidden_dropout_ratio=-1, num_hidden_layers=-1, initializer_range=-1, layer_norm_eps=1e-12,
                 local_rank=-1, seed=-1, fp16=False, pre_layer_norm=True, normalize_invertible=False,
                 gelu_checkpoint=False, adjust_init_range=True, attn_dropout_checkpoint=False, stochastic_mode=False,
                 return_tuple=False, training=True):
        super().__init__(batch_size, hidden_size, intermediate_size if intermediate_size > 0 else 4 * hidden_size,
                         heads, attn_dropout_ratio, hidden_dropout_ratio, num_hidden_layers, initializer_range)
        self.fp16 = fp16
        self.pre_layer_norm = pre_layer_norm
        self.local_rank = local_rank
        self.seed = seed
        self.normalize_invertible = normalize_invertible
        self.gelu_checkpoint = gelu_checkpoint
        self.adjust_init_range = adjust_init_range
        self.test_gemm = False
        self.layer_norm_eps = layer_norm_eps
        self.training = training
        self.is_grad_enabled = True
        self.attn_dropout_checkpoint = attn_dropout_checkpoint
        self.stochastic_mode = stochastic_mode
        self.return_tuple = return_tuple

    @classmethod
    def from_dict(cls, json_object):
        config = DeepSpeedTransformerConfig()
        for key, value in json_object.items():
            config.__dict__[key] = value
        return config

    @classmethod
    def from_json_file(cls, json_file):
        import json
        with open(json_file, "r", encoding="utf-16") as reader:
            return cls.from_dict(json.loads(reader.read()))


class DeepSpeedTransformerLayer(nn.Module):
    """One encoder block; forward(hidden_states [B, S, H], attention_mask [B, 1, 1, S] additive or None)."""
    layer_id = 0

    def __init__(self, config, initial_weights=None, initial_biases=None):
        super().__init__()
        self.config = config
        self.config.layer_id = DeepSpeedTransformerLayer.layer_id
        DeepSpeedTransformerLayer.layer_id += 1
        H, I = config.hidden_size, config.intermediate_size
        if initial_weights is None and initial_biases is None:
            self.attn_qkvw = nn.Parameter(torch.empty(3 * H, H))
            self.attn_qkvb = nn.Parameter(torch.empty(3 * H))
            self.attn_ow = nn.Parameter(torch.empty(H, H))
            self.attn_ob = nn.Parameter(torch.empty(H))
            self.attn_nw = nn.Parameter(torch.empty(H))
            self.attn_nb = nn.Parameter(torch.empty(H))
            self.inter_w = nn.Parameter(torch.empty(I, H))
            self.inter_b = nn.Parameter(torch.empty(I))
            self.output_w = nn.Parameter(torch.empty(H, I))
            self.output_b = nn.Parameter(torch.empty(H))
            self.norm_w = nn.Parameter(torch.empty(H))
            self.norm_b = nn.Parameter(torch.empty(H))
            self.init_transformer_weights(config.adjust_init_range)
        else:  # testing path of the reference: q, k, v, o, attn-norm, inter, output, norm
            w, b = initial_weights, initial_biases
            self.attn_qkvw = nn.Parameter(torch.cat([w[0].data, w[1].data, w[2].data]))
            self.attn_qkvb = nn.Parameter(torch.zeros(3 * H, dtype=w[0].dtype, device=w[0].device))
            self.attn_ow, self.attn_ob = w[3], b[3]
            self.attn_nw, self.attn_nb = w[4], b[4]
            self.inter_w, self.inter_b = w[5], b[5]
            self.output_w, self.output_b = w[6], b[6]
            self.norm_w, self.norm_b = w[7], b[7]
        if config.local_rank >= 0 and torch.cuda.is_available():
            torch.cuda.set_device(config.local_rank)

    def init_transformer_weights(self, adjust_init_range=False):
        std = self.config.initializer_range
        out_std = std / math.sqrt(2.0 * self.config.num_hidden_layers) if adjust_init_range else std
        with torch.no_grad():
            self.attn_qkvw.normal_(0.0, std)
            self.attn_qkvb.zero_()
            self.attn_ow.normal_(0.0, out_std)
            self.attn_ob.zero_()
            self.attn_nw.fill_(1.0)
            self.attn_nb.zero_()
            self.inter_w.normal_(0.0, std)
            self.inter_b.zero_()
            self.output_w.normal_(0.0, out_std)
            self.output_b.zero_()
            self.norm_w.fill_(1.0)
            self.norm_b.zero_()

    def _attention(self, qkv, B, S, mask):
        c = self.config
        nh = c.heads
        d = c.hidden_size // nh
        p_drop = c.attn_dropout_ratio if (self.training and c.attn_dropout_ratio > 0) else 0.0
        q, k, v = qkv.view(B, S, 3, nh, d).unbind(2)
        if p_drop == 0.0 and native_supported(q):
            # a right-padding key mask (the BERT case) runs the HIP kernel with per-sequence lengths
            lens = None if mask is None else self._mask_lengths(mask, S)
            if mask is None or lens is not None:
                return flash_attn(q.contiguous(), k.contiguous(), v.contiguous(), causal=False,
                                  seq_lens=lens).reshape(B * S, -1)
        qh, kh, vh = (t.transpose(1, 2) for t in (q, k, v))
        s = torch.matmul(qh, kh.transpose(-1, -2)).float() / math.sqrt(d)
        if mask is not None:
            s = s + mask.float()
        p = torch.softmax(s, -1)
        if p_drop > 0:
            p = F.dropout(p, p_drop, True)
        return torch.matmul(p.to(vh.dtype), vh).transpose(1, 2).reshape(B * S, -1)

    _mask_cache = (None, None, None)

    @classmethod
    def _mask_lengths(cls, mask, S):
        """Per-sequence lengths of a padding mask, computed once per mask tensor (every layer of a forward shares
        it) so the host sync of the prefix check is paid once per step, not once per layer."""
        key = (mask.data_ptr(), mask._version, tuple(mask.shape))
        if cls._mask_cache[0] != key:
            cls._mask_cache = (key, padding_mask_lengths(mask, S), None)
        return cls._mask_cache[1]

    def _dropout(self, x):
        r = self.config.hidden_dropout_ratio
        return F.dropout(x, r, True) if (self.training and r > 0) else x

    def forward(self, hidden_states, attention_mask=None, head_mask=None, layer_head_mask=None,
                encoder_hidden_states=None, encoder_attention_mask=None, past_key_value=None,
                output_attentions=False, grads=None):
        c = self.config
        c.is_grad_enabled = torch.is_grad_enabled()
        c.training = self.training
        B, S, H = hidden_states.shape
        x = hidden_states.reshape(B * S, H)
        eps = c.layer_norm_eps
        if c.pre_layer_norm:
            h = layer_norm(x, self.attn_nw, self.attn_nb, eps)
            a = self._attention(F.linear(h, self.attn_qkvw, self.attn_qkvb), B, S, attention_mask)
            a = self._dropout(F.linear(a, self.attn_ow, self.attn_ob))
            h, x1 = layer_norm(a, self.norm_w, self.norm_b, eps, residual=x)  # x1 = x + attn
            f = bias_act(F.linear(h, self.inter_w), self.inter_b, "gelu_tanh")
            out = x1 + self._dropout(F.linear(f, self.output_w, self.output_b))
        else:
            a = self._attention(F.linear(x, self.attn_qkvw, self.attn_qkvb), B, S, attention_mask)
            a = self._dropout(F.linear(a, self.attn_ow, self.attn_ob))
            h, _ = layer_norm(a, self.attn_nw, self.attn_nb, eps, residual=x)
            f = bias_act(F.linear(h, self.inter_w), self.inter_b, "gelu_tanh")
            o = self._dropout(F.linear(f, self.output_w, self.output_b))
            out, _ = layer_norm(o, self.norm_w, self.norm_b, eps, residual=h)
        out = out.view(B, S, H)
        return (out, ) if c.return_tuple else out
