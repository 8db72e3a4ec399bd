"""Token embedding whose weight gradient is scatter-added in place (csrc/kernels/token_ops.hip embed_bwd_kernel).

The framework's default ``nn.Embedding`` backward sorts the ids, reduces duplicates into a DENSE [V, D]
gradient (fill + compute_grad_weight + sum_and_scatter) and AccumulateGrad then adds that whole tensor into
``.grad`` -- for Llama-3 (V=128256, D=4096) three passes over 1 GB per micro-step. Here the ids are sorted
once and one HIP workgroup per distinct id adds its tokens' rows straight into the parameter's gradient
buffer (the flat ZeRO buffer), touching only the rows that occur. Reference counterpart: the embedding of
every model trained through ``deepspeed.initialize`` (the reference uses the framework kernel).

CPU tensors use ``index_add_`` (the numerics reference of the tests).
"""
import types

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import native


def embedding_grad_add_(grad, ids, dy, padding_idx=None):
    """grad[ids[t]] += dy[t] for every token t (rows equal to ``padding_idx`` skipped); deterministic."""
    V, D = grad.shape
    ids = ids.reshape(-1)
    dy = dy.reshape(-1, D)
    if native.use_native(grad) and D % 8 == 0 and dy.dtype == grad.dtype and \
            grad.dtype in (torch.float32, torch.bfloat16, torch.float16) and grad.is_contiguous():
        dy = dy.contiguous()
        srt, perm = torch.sort(ids.to(torch.int64), stable=True)
        pad = -1 if padding_idx is None else int(padding_idx) % V
        native.check(native.kernels().hds_embed_bwd(native.dt(grad), dy.data_ptr(), srt.data_ptr(), perm.data_ptr(),
                                                    grad.data_ptr(), ids.numel(), D, V, pad, native.stream()),
                     "embed_bwd")
        return grad
    if padding_idx is not None:
        keep = ids != (int(padding_idx) % V)
        ids, dy = ids[keep], dy[keep]
    grad.index_add_(0, ids.to(torch.int64), dy.to(grad.dtype))
    return grad


class EmbeddingFunction(torch.autograd.Function):

    @staticmethod
    def forward(ctx, ids, weight, padding_idx):
        ctx.save_for_backward(ids)
        ctx.weight = weight  # the Parameter object: under ZeRO-3 its storage is re-gathered for backward
        ctx.shape = tuple(weight.shape)
        ctx.padding_idx = padding_idx
        return F.embedding(ids, weight, padding_idx)

    @staticmethod
    def backward(ctx, dy):
        from ..runtime.zero.linear import grad_accumulator
        (ids, ) = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None, None
        g = grad_accumulator(ctx.weight, dy.dtype)
        if g is not None:
            embedding_grad_add_(g.view(ctx.shape), ids, dy, ctx.padding_idx)
            return None, None, None
        dw = torch.zeros(ctx.shape, dtype=dy.dtype, device=dy.device)
        return None, embedding_grad_add_(dw, ids, dy, ctx.padding_idx), None


def _emb_forward(self, ids):
    return EmbeddingFunction.apply(ids, self.weight, self.padding_idx)


def wrap_embeddings(module, only=None):
    """Route plain dense nn.Embedding modules under ``module`` (or those whose weight id is in ``only``) through
    :class:`EmbeddingFunction` (instance-level forward override)."""
    n = 0
    for m in module.modules():
        if isinstance(m, nn.Embedding) and not getattr(m, "_hds_emb", False) and not m.sparse and \
                m.max_norm is None and not m.scale_grad_by_freq and (only is None or id(m.weight) in only):
            m.forward = types.MethodType(_emb_forward, m)
            m._hds_emb = True
            n += 1
    return n
