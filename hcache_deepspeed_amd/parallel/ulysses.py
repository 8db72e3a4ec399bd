"""Ulysses sequence parallelism: all-to-all head<->sequence re-sharding around any local attention.

Reference parity: sequence/layer.py (``DistributedAttention`` :311-420, ``_SeqAllToAll``, uneven heads / GQA
:111-218) and the engine's DP x SP mesh (__init__.py:153-162, ZeRO over the seq-data-parallel group).

On a fully connected 8x MI355X xGMI mesh one ``all_to_all_single`` drives all 7 links of every GPU at
once, so the per-GPU volume (M/P per tensor) moves at the aggregate link bandwidth -- Ulysses is the
natural long-context strategy on this fabric (ring attention is per-link bound).

For the Llama model the all-to-all is applied to the FUSED QKV projection output: heads are permuted
so every rank's slice holds its own q | k | v heads contiguously, one all-to-all moves all three, RoPE +
FlashAttention run on the full sequence for H/P heads, and one all-to-all brings the output back.
"""
import torch

from .. import comm as dist


def _a2a(x, group):
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x.contiguous(), group=group)
    return out


def seq_to_head(x, group, B):
    """[B*S/P, NH, D] (local tokens, all heads) -> [B*S, NH/P, D] (all tokens, my heads)."""
    P = dist.get_world_size(group)
    T, NH, D = x.shape
    Sl = T // B
    hg = NH // P
    # [B, Sl, P, hg, D] -> [P, B, Sl, hg, D]: chunk p goes to rank p
    send = x.view(B, Sl, P, hg, D).permute(2, 0, 1, 3, 4).contiguous()
    recv = _a2a(send, group)  # [P(src = seq chunk), B, Sl, hg, D]
    return recv.permute(1, 0, 2, 3, 4).reshape(B * P * Sl, hg, D)


def head_to_seq(x, group, B):
    """[B*S, NH/P, D] -> [B*S/P, NH, D] (inverse of seq_to_head)."""
    P = dist.get_world_size(group)
    T, hg, D = x.shape
    S = T // B
    Sl = S // P
    send = x.view(B, P, Sl, hg, D).permute(1, 0, 2, 3, 4).contiguous()  # chunk p = seq chunk p -> rank p
    recv = _a2a(send, group)  # [P(src = head group), B, Sl, hg, D]
    return recv.permute(1, 2, 0, 3, 4).reshape(B * Sl, P * hg, D)


class _SeqToHead(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, group, B):
        ctx.group, ctx.B = group, B
        return seq_to_head(x, group, B)

    @staticmethod
    def backward(ctx, g):
        return head_to_seq(g.contiguous(), ctx.group, ctx.B), None, None


class _HeadToSeq(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, group, B):
        ctx.group, ctx.B = group, B
        return head_to_seq(x, group, B)

    @staticmethod
    def backward(ctx, g):
        return seq_to_head(g.contiguous(), ctx.group, ctx.B), None, None


class _SeqAllToAll(torch.autograd.Function):
    """Reference-compatible 4D all-to-all: [B, S/P, H, D] <-> [B, S, H/P, D] (scatter_idx=2, gather_idx=1)."""

    @staticmethod
    def forward(ctx, group, x, scatter_idx, gather_idx):
        ctx.group, ctx.s, ctx.g = group, scatter_idx, gather_idx
        B = x.shape[0]
        if scatter_idx == 2:
            y = seq_to_head(x.reshape(-1, x.shape[2], x.shape[3]), group, B)
            return y.view(B, -1, y.shape[1], y.shape[2])
        y = head_to_seq(x.reshape(-1, x.shape[2], x.shape[3]), group, B)
        return y.view(B, -1, y.shape[1], y.shape[2])

    @staticmethod
    def backward(ctx, g):
        return None, _SeqAllToAll.apply(ctx.group, g, ctx.g, ctx.s), None, None


class DistributedAttention(torch.nn.Module):
    """Wrap a local attention ``fn(q, k, v, *args)`` on [B, S, H, D] tensors into Ulysses SP."""

    def __init__(self, local_attention, sequence_process_group, scatter_idx=2, gather_idx=1, sp_stream=None):
        super().__init__()
        self.local_attn = local_attention
        self.spg = sequence_process_group
        self.scatter_idx, self.gather_idx = scatter_idx, gather_idx

    def forward(self, query, key, value, *args, **kwargs):
        q = _SeqAllToAll.apply(self.spg, query, self.scatter_idx, self.gather_idx)
        k = _SeqAllToAll.apply(self.spg, key, self.scatter_idx, self.gather_idx)
        v = _SeqAllToAll.apply(self.spg, value, self.scatter_idx, self.gather_idx)
        ctx = self.local_attn(q, k, v, *args, **kwargs)
        return _SeqAllToAll.apply(self.spg, ctx, self.gather_idx, self.scatter_idx)


def qkv_head_permutation(n_q, n_kv, P):
    """Index order putting rank r's (q, k, v) heads contiguously: [q_0 k_0 v_0 | q_1 k_1 v_1 | ...]."""
    lq, lkv = n_q // P, n_kv // P
    idx = []
    for r in range(P):
        idx += list(range(r * lq, (r + 1) * lq))
        idx += list(range(n_q + r * lkv, n_q + (r + 1) * lkv))
        idx += list(range(n_q + n_kv + r * lkv, n_q + n_kv + (r + 1) * lkv))
    return idx


def ulysses_qkv(qkv, n_q, n_kv, group, B):
    """[B*S/P, n_q+2n_kv, D] -> [B*S, (n_q+2n_kv)/P, D] with my heads in q|k|v order (differentiable)."""
    P = dist.get_world_size(group)
    assert n_q % P == 0 and n_kv % P == 0, f"Ulysses needs heads divisible by sp={P} (q={n_q}, kv={n_kv})"
    perm = torch.tensor(qkv_head_permutation(n_q, n_kv, P), device=qkv.device)
    return _SeqToHead.apply(qkv.index_select(1, perm), group, B)


def ulysses_out(o, group, B):
    """[B*S, n_q/P, D] -> [B*S/P, n_q, D] (differentiable)."""
    return _HeadToSeq.apply(o, group, B)


def enable_sequence_parallel(model, group):
    """Turn on Ulysses for every LlamaAttention in ``model``."""
    from ..models.llama import LlamaAttention
    n = 0
    P = dist.get_world_size(group)
    for m in model.modules():
        if isinstance(m, LlamaAttention):
            m.sp_group = group
            n += 1
        if hasattr(m, "rope") and hasattr(m, "layers"):
            m._hds_sp_size = P  # RoPE tables must cover the full (gathered) sequence
    model._hds_sp_group = group
    return n
