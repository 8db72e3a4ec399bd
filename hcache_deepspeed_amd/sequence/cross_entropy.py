"""Vocab-and-sequence-parallel cross entropy for Ulysses (reference deepspeed/sequence/cross_entropy.py
``vocab_sequence_parallel_cross_entropy``): every SP rank holds the logits of its slice of the sequence,
[S/P, B, V]; the per-token losses of the whole sequence, [S, B], are all-gathered so every rank sees the same loss.

Here the per-token loss and d(loss)/d(logits) come from one pass of the HIP cross-entropy kernel
(ops/cross_entropy.py, csrc/kernels/xent.hip), which writes the unscaled gradient over a copy of the logits in the
forward; the backward only scales this rank's slice by the incoming gradient. The reference keeps a softmax copy and
edits it in the backward -- the same V-sized buffer, but a second pass.
"""
import torch

from .. import comm as dist
from ..ops.cross_entropy import cross_entropy


class _VocabSequenceParallelCE(torch.autograd.Function):

    @staticmethod
    def forward(ctx, logits, target, sp_group):
        with torch.enable_grad():
            lg = logits.detach().requires_grad_(True)
            loss = cross_entropy(lg, target, reduction="none")  # [S/P, B]; grad graph kept for the backward
        ctx.lg, ctx.loss = lg, loss
        P = dist.get_world_size(sp_group)
        ctx.P, ctx.r = P, dist.get_rank(sp_group)
        out = loss.new_empty((loss.shape[0] * P, ) + tuple(loss.shape[1:]))
        dist.all_gather_into_tensor(out, loss.detach().contiguous(), group=sp_group)
        return out.to(logits.dtype)

    @staticmethod
    def backward(ctx, g):
        n = g.shape[0] // ctx.P
        mine = g[ctx.r * n:(ctx.r + 1) * n].float()
        (dlogits, ) = torch.autograd.grad(ctx.loss, ctx.lg, mine)
        ctx.lg = ctx.loss = None
        return dlogits, None, None


def vocab_sequence_parallel_cross_entropy(vocab_parallel_logits, target, sp_group):
    """logits [S/P, B, V], target [S/P, B] -> per-token loss [S, B] of the full sequence (same on every SP rank)."""
    return _VocabSequenceParallelCE.apply(vocab_parallel_logits, target, sp_group)
