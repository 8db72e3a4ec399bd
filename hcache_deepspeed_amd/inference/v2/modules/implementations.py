"""Registered inference-v2 module implementations on the MI355X kernels
(reference inference/v2/modules/implementations/*: dense_blocked_attention, blas_fp_linear, quantized_linear
(wf6af16), cutlass_multi_gemm_moe, cuda_pre_rms / cuda_pre_ln / cuda_post_ln, ragged_embedding, ragged_unembed).

* attention: fused RoPE + paged-KV scatter and paged FlashAttention (csrc/kernels/paged_attn.hip, MFMA);
* linear: bf16 GEMM on hipBLASLt with the bias/activation epilogue in the HIP activation kernels; FP6 (e3m2) and
  INT8/INT4 weight-only variants read the packed weight straight from HBM at decode sizes (HIP GEMVs) and
  dequantize once per call for prefill-sized batches;
* MoE: sync-free top-k assignment + dropless grouped GEMM (csrc/kernels/grouped_gemm.hip);
* norms: the fused residual-add + RMSNorm / LayerNorm kernels (csrc/kernels/norm.hip).
"""
import torch
import torch.nn.functional as F

from .... import comm as dist
from ....ops.activations import bias_act, glu
from ....ops.grouped_gemm import moe_ffn_dropless
from ....ops.moe import moe_combine, moe_dispatch, topk_assign, topk_route
from ....ops.norm import layer_norm, rms_norm
from ....ops.paged import kv_rope_scatter, paged_attention
from ....ops.quantizer import fp6_linear, int_linear, quantize, quantize_minifloat
from .interfaces import (DSEmbeddingBase, DSEmbeddingRegistry, DSLinearBase, DSLinearRegistry, DSMoEBase,
                         DSMoERegistry, DSPostNormBase, DSPostNormRegistry, DSPreNormBase, DSPreNormRegistry,
                         DSSelfAttentionBase, DSSelfAttentionRegistry, DSUnembedBase, DSUnembedRegistry)

_PLAIN_ACTS = ("gelu", "gelu_tanh", "relu", "silu")


def _act_tail(y, bias, activation):
    """bias + activation epilogue shared by every linear implementation."""
    if activation == "identity":
        return y if bias is None else y + bias
    if activation.endswith("_glu"):
        return glu(y if bias is None else y + bias, activation[:-4])
    return bias_act(y, bias, activation)


def _supports_act(a):
    return a == "identity" or a in _PLAIN_ACTS or (a.endswith("_glu") and a[:-4] in _PLAIN_ACTS)


# ---------------------------------------------------------------------------------------------------------------
@DSSelfAttentionRegistry.register_module
class DSDenseBlockedAttention(DSSelfAttentionBase):

    @staticmethod
    def name():
        return "dense_blocked_attention"

    @staticmethod
    def supports_config(c):
        return c.n_heads_q % c.n_heads_kv == 0 and c.head_size % 16 == 0 and c.head_size <= 256

    def forward(self, qkv, cache, batch, cos, sin):
        c = self._config
        T = qkv.shape[0]
        nq, nkv, D = c.n_heads_q, c.n_heads_kv, c.head_size
        kv_rope_scatter(qkv, cache, batch.tok_seq, batch.tok_pos, batch.block_tables, cos, sin, nq, nkv,
                        do_rope=c.positional_embedding_type != "none" and cos is not None, rotary_dim=c.rotary_dim)
        o = paged_attention(qkv[:, :nq], cache, batch.atoms, batch.n_atoms, batch.seq_meta, batch.block_tables, nq,
                            nkv, c.scale_factor, c.sliding_window, batch.seq_meta_host, batch.tables_host,
                            decode=T == batch.current_sequences)
        return o.reshape(T, nq * D)


# ---------------------------------------------------------------------------------------------------------------
@DSLinearRegistry.register_module
class BlasFPLinear(DSLinearBase):

    @staticmethod
    def name():
        return "blas_fp_linear"

    @staticmethod
    def supports_config(c):
        return c.quantization_mode is None and _supports_act(c.activation)

    def forward(self, x, w, b=None):
        a = self._config.activation
        from ....ops.gemv import linear  # decode-sized ragged batches (<= 8 tokens) on the HIP GEMV
        if a == "identity" or a.endswith("_glu"):
            return _act_tail(linear(x, w, b), None, a)
        return bias_act(linear(x, w), b, a)


class _PackedWeight:
    """Weight-only quantized [out, in] matrix (groups along ``in``)."""

    def __init__(self, q, scales, out_features, in_features, group_size):
        self.q, self.scales = q, scales
        self.out_features, self.in_features, self.group_size = out_features, in_features, group_size
        self.shape = (out_features, in_features)

    def nbytes(self):
        return self.q.numel() * self.q.element_size() + self.scales.numel() * 4


def _group(c, in_features):
    g = c.group_size
    while in_features % g:
        g //= 2
    return g


@DSLinearRegistry.register_module
class QuantizedWf6Af16Linear(DSLinearBase):
    """FP6 (e3m2) weights, bf16 activations: the reference's ``quantized_wf6af16_linear``."""

    @staticmethod
    def name():
        return "quantized_wf6af16_linear"

    @staticmethod
    def supports_config(c):
        return c.quantization_mode == "wf6af16" and _supports_act(c.activation) and c.in_channels % 16 == 0

    def transform_param(self, w):
        if isinstance(w, _PackedWeight) or w is None:
            return w
        out_f, in_f = w.shape
        g = _group(self._config, in_f)
        q, s = quantize_minifloat(w.contiguous(), g, 6, 2)
        return _PackedWeight(q, s, out_f, in_f, g)

    def forward(self, x, w, b=None):
        y = fp6_linear(x, w.q, w.scales, w.out_features, w.in_features, w.group_size, 2)
        return _act_tail(y, b, self._config.activation)


@DSLinearRegistry.register_module
class QuantizedIntLinear(DSLinearBase):
    """Symmetric group-wise INT8 / INT4 weights, bf16 activations (inference v1's int8 weight path in v2)."""

    @staticmethod
    def name():
        return "quantized_int_linear"

    @staticmethod
    def supports_config(c):
        return c.quantization_mode in ("int8", "int4") and _supports_act(c.activation) and c.in_channels % 16 == 0

    def _bits(self):
        return 8 if self._config.quantization_mode == "int8" else 4

    def transform_param(self, w):
        if isinstance(w, _PackedWeight) or w is None:
            return w
        out_f, in_f = w.shape
        g = _group(self._config, in_f)
        q, s, _ = quantize(w.contiguous(), g, self._bits(), True)
        return _PackedWeight(q, s, out_f, in_f, g)

    def forward(self, x, w, b=None):
        y = int_linear(x, w.q, w.scales, w.out_features, w.in_features, w.group_size, self._bits())
        return _act_tail(y, b, self._config.activation)


# ---------------------------------------------------------------------------------------------------------------
@DSMoERegistry.register_module
class GroupedGemmMoE(DSMoEBase):
    """Top-k MoE without token dropping. GPU bf16: sync-free routing + two HIP grouped GEMMs over the
    expert-contiguous rows; elsewhere: capacity slots + batched expert GEMMs."""

    @staticmethod
    def name():
        return "grouped_gemm_moe"

    @staticmethod
    def supports_config(c):
        return c.activation.endswith("_glu") and 1 <= c.top_k <= c.n_experts

    def forward(self, x, router_w, w13, w2):
        c = self._config
        act = c.activation[:-4]
        T, H = x.shape
        logits = F.linear(x.float(), router_w.float())
        if x.is_cuda and x.dtype == torch.bfloat16 and H % 128 == 0 and w2.shape[2] % 128 == 0:
            expert, pos, w, counts = topk_assign(logits, c.top_k, normalize=c.normalize_scores)
            return moe_ffn_dropless(x, expert, pos, w, counts, w13, w2, lambda h: glu(h, act))
        E = logits.shape[-1]
        expert, pos, w, C, _, _ = topk_route(logits, c.top_k, 1.0, 1, drop_tokens=False, use_rts=False,
                                             normalize=c.normalize_scores, training=False)
        disp = moe_dispatch(x, expert, pos, E, C).view(E, C, H)
        from ....parallel.moe import expert_linear  # per-expert 2-D GEMMs on the GPU (see its docstring)
        with torch.no_grad():
            h = expert_linear(disp, w13)
            y = expert_linear(glu(h.reshape(E * C, -1), act).view(E, C, -1), w2)
        return moe_combine(y.reshape(E * C, H), expert, pos, w, C)


# ---------------------------------------------------------------------------------------------------------------
@DSPreNormRegistry.register_module
class DSPreRMSNorm(DSPreNormBase):

    @staticmethod
    def name():
        return "ds_pre_rms"

    @staticmethod
    def supports_config(c):
        return c.type == "rms"

    def forward(self, residual, hidden_in, gamma, beta=None):
        if hidden_in is None:
            return residual, rms_norm(residual, gamma, self._config.eps)
        y, r = rms_norm(hidden_in, gamma, self._config.eps, residual)
        return r, y


@DSPreNormRegistry.register_module
class DSPreLayerNorm(DSPreNormBase):

    @staticmethod
    def name():
        return "ds_pre_ln"

    @staticmethod
    def supports_config(c):
        return c.type == "layer"

    def forward(self, residual, hidden_in, gamma, beta=None):
        if hidden_in is None:
            return residual, layer_norm(residual, gamma, beta, self._config.eps)
        y, r = layer_norm(hidden_in, gamma, beta, self._config.eps, residual)
        return r, y


@DSPostNormRegistry.register_module
class DSPostLayerNorm(DSPostNormBase):

    @staticmethod
    def name():
        return "ds_post_ln"

    @staticmethod
    def supports_config(c):
        return c.type in ("layer", "rms")

    def forward(self, residual, hidden_in, gamma, beta=None):
        if self._config.type == "rms":
            y, _ = rms_norm(hidden_in, gamma, self._config.eps, residual)
        else:
            y, _ = layer_norm(hidden_in, gamma, beta, self._config.eps, residual)
        return y


# ---------------------------------------------------------------------------------------------------------------
@DSEmbeddingRegistry.register_module
class RaggedEmbedding(DSEmbeddingBase):

    @staticmethod
    def name():
        return "ragged_embedding"

    def forward(self, batch, word_embeddings, position_embeddings=None):
        h = F.embedding(batch.input_ids, word_embeddings)
        if position_embeddings is not None:
            h = h + F.embedding(batch.tok_pos.long() + self._config.positional_offset, position_embeddings)
        return h


@DSUnembedRegistry.register_module
class RaggedUnembed(DSUnembedBase):
    """Gathers each sequence's last token, applies the final norm (fused residual add) and the vocab GEMM; under
    TP the vocab is sharded by rows and the shards are all-gathered."""

    @staticmethod
    def name():
        return "ragged_unembed"

    def forward(self, hidden, residual, batch, lm_head, lm_head_b, final_w, final_b, norm_eps=1e-5, tp_group=None,
                vocab=None):
        idx = batch.last_token_idx
        if final_w is not None:
            if self._config.norm_type == "rms":
                hl, _ = rms_norm(hidden[idx], final_w, norm_eps, residual[idx])
            else:
                hl, _ = layer_norm(hidden[idx], final_w, final_b, norm_eps, residual[idx])
        else:
            hl = hidden[idx] + residual[idx]
        logits = F.linear(hl, lm_head, lm_head_b)
        tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        if tp > 1:
            parts = [torch.empty_like(logits) for _ in range(tp)]
            dist.all_gather(parts, logits, group=tp_group)
            logits = torch.cat(parts, -1)[:, :vocab]
        return logits
