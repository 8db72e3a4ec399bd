"""Domino: tensor-parallel training that hides the TP all-reduces behind compute of the other half-batch.

Reference parity: runtime/domino/transformer.py (``DominoTransformerLayer`` :250-408 -- each micro-batch is
split into two halves; the async all-reduce of half 0's attention / MLP output overlaps half 1's compute and
vice versa; ``DominoTransformer`` :411) and runtime/domino/async_linear.py (``DominoAsyncColumnParallelLinear``:
the column-parallel backward all-reduce of dX is issued async and waited late).

MI355X design: every TP all-reduce is an RCCL collective over the dedicated xGMI link pairs, issued with
``async_op=True`` so it runs on RCCL's own HIP stream; ``work.wait()`` only inserts a stream dependency, so
the other half's kernels that were enqueued in between execute concurrently with the all-reduce. Applied to
this framework's fused Llama block (fused QKV / gate-up GEMMs, fused residual RMSNorm):

    fwd per layer:  attn(h0) -> AR0 |  attn(h1) -> AR1 | wait AR0, mlp(h0) -> AR0' | wait AR1, mlp(h1) -> AR1'
    bwd:            column-parallel dX all-reduce runs async under the dW GEMM (parallel/tp._ColumnParallelFn).

Use :func:`enable_domino` on a model whose linears were sharded by AutoTP (``tensor_parallel.autotp_size``).
"""
import torch
import torch.nn.functional as F

from .. import comm as dist
from ..ops.activations import glu
from ..ops.attention import qkv_attention


class _AsyncAllReduceStart(torch.autograd.Function):
    """fwd: launch an async SUM all-reduce of ``x`` (in place) and park the handle; bwd: identity
    (row-parallel semantics: the gradient of a replicated sum is replicated)."""

    @staticmethod
    def forward(ctx, x, group, slot):
        x = x.contiguous()
        slot["work"] = dist.all_reduce(x, group=group, async_op=True) if dist.get_world_size(group) > 1 else None
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None, None


class _AsyncAllReduceWait(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, slot):
        w = slot.pop("work", None)
        if w is not None:
            w.wait()
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g, None


def _ar_start(x, group):
    slot = {}
    return _AsyncAllReduceStart.apply(x, group, slot), slot


def _ar_wait(x, slot):
    return _AsyncAllReduceWait.apply(x, slot)


def _column(x, lin):
    from .tp import _ColumnParallelFn, LinearLayer
    if isinstance(lin, LinearLayer):
        return _ColumnParallelFn.apply(x, lin.weight, lin.bias, lin.tp_group)
    return lin(x)


def _row_partial(x, lin):
    """Row-parallel GEMM WITHOUT its all-reduce (Domino issues that async)."""
    return F.linear(x, lin.weight)


def _row_bias(y, lin):
    return y + lin.bias if getattr(lin, "bias", None) is not None else y


def _attn_partial(layer, x, cos, sin, seq_len):
    a = layer.self_attn
    T = x.shape[0]
    qkv = _column(x, a.qkv_proj).view(T, a.n_q + 2 * a.n_kv, a.d)
    o = qkv_attention(qkv, a.n_q, a.n_kv, cos, sin, seq_len=seq_len, causal=True, window=a.cfg.sliding_window)
    return _row_partial(o, a.o_proj)


def _mlp_partial(layer, x):
    m = layer.mlp
    return _row_partial(glu(_column(x, m.gate_up_proj), m.act), m.down_proj)


def domino_layer_forward(layer, hs, residuals, cos, sin, seq_len, group):
    """One decoder layer on two half-batches with the TP all-reduces overlapped (reference :320-408)."""
    (h0, h1), (r0, r1) = hs, residuals
    ln1, ln2 = layer.input_layernorm, layer.post_attention_layernorm

    def pre(h, r):
        if r is None:
            return ln1(h), h
        return ln1(h, r)

    x0, r0 = pre(h0, r0)
    a0, s0 = _ar_start(_attn_partial(layer, x0, cos, sin, seq_len), group)
    x1, r1 = pre(h1, r1)
    a1, s1 = _ar_start(_attn_partial(layer, x1, cos, sin, seq_len), group)

    a0 = _row_bias(_ar_wait(a0, s0), layer.self_attn.o_proj)
    x0, r0 = ln2(a0, r0)
    m0, t0 = _ar_start(_mlp_partial(layer, x0), group)

    a1 = _row_bias(_ar_wait(a1, s1), layer.self_attn.o_proj)
    x1, r1 = ln2(a1, r1)
    m1, t1 = _ar_start(_mlp_partial(layer, x1), group)

    m0 = _row_bias(_ar_wait(m0, t0), layer.mlp.down_proj)
    m1 = _row_bias(_ar_wait(m1, t1), layer.mlp.down_proj)
    return (m0, m1), (r0, r1)


def domino_decoder_forward(model, h, cos, sin, seq_len, B):
    """Run every decoder layer of a LlamaModel with Domino overlap; ``h``: [B*S, H] embeddings."""
    group = model._domino_group
    b0 = B // 2
    hs = (h[:b0 * seq_len], h[b0 * seq_len:])
    rs = (None, None)
    for layer in model.layers:
        hs, rs = domino_layer_forward(layer, hs, rs, cos, sin, seq_len, group)
    return torch.cat(hs, 0), torch.cat(rs, 0)


def enable_domino(model, group=None):
    """Switch a (TP-sharded) LlamaForCausalLM / LlamaModel to Domino execution. Micro-batches with an odd batch
    size (or varlen / SP / FPDT batches) fall back to the plain TP path."""
    from ..models.llama import LlamaModel
    from .tp import LinearAllreduce
    if group is None:
        for m in model.modules():
            if isinstance(m, LinearAllreduce):
                group = m.tp_group
                break
    n = 0
    for m in model.modules():
        if isinstance(m, LlamaModel):
            m._domino_group = group
            n += 1
    assert n, "enable_domino: no LlamaModel found"
    return model


class DominoTransformer(torch.nn.Module):
    """Reference-named wrapper: ``DominoTransformer(model)`` enables Domino on a TP-sharded Llama model."""

    def __init__(self, model, group=None):
        super().__init__()
        self.module = enable_domino(model, group)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)
