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


def shard_sizes(n, P):
    """Uneven split of ``n`` heads over ``P`` ranks, larger shards first (reference get_shard_size_list)."""
    return [n // P + (1 if r < n % P else 0) for r in range(P)]


def ulysses_head_plan(n_q, n_kv, P):
    """Per rank r: (q head indices, kv head indices) of its slice. With at least one kv head per rank, whole GQA
    groups are split over the ranks (unevenly when ``n_kv % P``). With fewer kv heads than ranks the query heads are
    split (unevenly when ``n_q % P``) and each rank receives the kv heads its query heads use (GQA group size
    ``n_q // n_kv``): kv heads are REPLICATED. A rank whose query heads form equal
    runs per kv head keeps GQA locally (one copy per kv head, local group size = run length); otherwise its kv
    heads are expanded to one per query head (local MHA). Either way the local attention's q head i uses kv head
    i // (len(q) // len(kv)), the contract of the FlashAttention kernels."""
    assert n_q % n_kv == 0, (n_q, n_kv)
    G = n_q // n_kv
    if n_kv >= P:  # whole GQA groups per rank (uneven group counts): no kv head is replicated
        plan, a = [], 0
        for n in shard_sizes(n_kv, P):
            plan.append((list(range(a * G, (a + n) * G)), list(range(a, a + n))))
            a += n
        return plan
    sizes = shard_sizes(n_q, P)
    assert min(sizes) > 0, f"Ulysses needs at least one query head per rank (q={n_q}, sp={P})"
    plan, a = [], 0
    for n in sizes:
        q = list(range(a, a + n))
        a += n
        kv_of = [h // G for h in q]
        runs = []
        for k in kv_of:
            if runs and runs[-1][0] == k:
                runs[-1][1] += 1
            else:
                runs.append([k, 1])
        if len({c for _, c in runs}) == 1:
            kv = [k for k, _ in runs]
        else:
            kv = kv_of  # unequal runs: one kv copy per query head
        plan.append((q, kv))
    return plan


class _A2A(torch.autograd.Function):
    """all_to_all_single of a flat tensor with per-rank split sizes (elements); backward swaps the splits."""

    @staticmethod
    def forward(ctx, x, in_splits, out_splits, group):
        ctx.in_splits, ctx.out_splits, ctx.group = in_splits, out_splits, group
        out = x.new_empty(sum(out_splits))
        dist.all_to_all_single(out, x.contiguous(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        return _A2A.apply(g.contiguous(), ctx.out_splits, ctx.in_splits, ctx.group), None, None, None


def seq_to_heads(x, group, B, send_heads):
    """[B*S/P, NH, D] local tokens, all heads -> [B*S, len(send_heads[me]), D]: every rank receives ITS head list
    (lists may differ in length and overlap) for the whole sequence. Differentiable (gradients of a head sent to
    several ranks are summed by index_select's backward)."""
    P = dist.get_world_size(group)
    me = dist.get_rank(group)
    T, NH, D = x.shape
    Sl = T // B
    idx = torch.tensor([h for r in range(P) for h in send_heads[r]], device=x.device, dtype=torch.long)
    send = x.index_select(1, idx).permute(1, 0, 2).reshape(-1)  # [heads for r0 | r1 | ...] x [T, D]
    in_splits = [len(send_heads[r]) * T * D for r in range(P)]
    n_me = len(send_heads[me])
    out = _A2A.apply(send, in_splits, [n_me * T * D] * P, group)  # [P(src = seq chunk), n_me, B, Sl, D]
    return out.view(P, n_me, B, Sl, D).permute(2, 0, 3, 1, 4).reshape(B * P * Sl, n_me, D)


def heads_to_seq(o, group, B, head_counts):
    """[B*S, head_counts[me], D] (all tokens, my heads) -> [B*S/P, sum(head_counts), D] (my tokens, all heads in
    rank order). Differentiable."""
    P = dist.get_world_size(group)
    me = dist.get_rank(group)
    T, n_me, D = o.shape
    S = T // B
    Sl = S // P
    send = o.view(B, P, Sl, n_me, D).permute(1, 3, 0, 2, 4).reshape(-1)  # [P(dst = seq chunk), n_me, B, Sl, D]
    per = B * Sl * D
    out = _A2A.apply(send, [n_me * per] * P, [head_counts[r] * per for r in range(P)], group)
    parts = out.split([head_counts[r] * per for r in range(P)])
    full = torch.cat([p.view(head_counts[r], B, Sl, D) for r, p in enumerate(parts)], 0)  # [NH, B, Sl, D]
    return full.permute(1, 2, 0, 3).reshape(B * Sl, sum(head_counts), D)


class _SeqAllToAll3(torch.autograd.Function):
    """q, k, v all-to-alls ISSUED TOGETHER (async), then waited: the reference's q/k/v overlap on ``sp_stream``
    (sequence/layer.py:337-417). On RCCL the three collectives queue back to back on the communicator's stream
    instead of each waiting for the previous one's completion on the host."""

    @staticmethod
    def forward(ctx, group, B, q, k, v):
        ctx.group, ctx.B = group, B
        ctx.shapes = [t.shape for t in (q, k, v)]
        return _a2a_many([t.reshape(-1, t.shape[2], t.shape[3]) for t in (q, k, v)], group, B, True)

    @staticmethod
    def backward(ctx, gq, gk, gv):
        gs = _a2a_many([g.reshape(-1, g.shape[2], g.shape[3]) for g in (gq, gk, gv)], ctx.group, ctx.B, False)
        return (None, None) + tuple(g.reshape(s) for g, s in zip(gs, ctx.shapes))


def _a2a_many(xs, group, B, to_heads):
    """Even-head 4D re-sharding of several [T, H, D] tensors with every all-to-all in flight before the first wait."""
    P = dist.get_world_size(group)
    works, outs, post = [], [], []
    for x in xs:
        T, H, D = x.shape
        if to_heads:
            Sl, hg = T // B, H // P
            send = x.view(B, Sl, P, hg, D).permute(2, 0, 1, 3, 4).contiguous()
        else:
            S = T // B
            Sl, hg = S // P, H
            send = x.view(B, P, Sl, hg, D).permute(1, 0, 2, 3, 4).contiguous()
        out = torch.empty_like(send)
        works.append(dist.all_to_all_single(out, send, group=group, async_op=True))
        outs.append(out)
        post.append((B, Sl, hg, D))
    res = []
    for w, out, (B_, Sl, hg, D) in zip(works, outs, post):
        if w is not None:
            w.wait()
        if to_heads:
            y = out.permute(1, 0, 2, 3, 4).reshape(B_, P * Sl, hg, D)
        else:
            y = out.permute(1, 2, 0, 3, 4).reshape(B_, Sl, P * hg, D)
        res.append(y)
    return tuple(res)


class DistributedAttention(torch.nn.Module):
    """Wrap a local attention ``fn(q, k, v, *args)`` on [B, S, H, D] tensors into Ulysses SP.

    Heads need not divide the SP size, and k / v may have fewer heads than ranks (GQA): then the heads are split
    unevenly and kv heads replicated per ``ulysses_head_plan``, and the local attention receives q with its local
    query heads and k / v with the kv heads those use. With even heads the q / k / v all-to-alls are issued
    together before the first wait (``sp_stream`` given or not -- there is nothing to gain from serialising them)."""

    def __init__(self, local_attention, sequence_process_group, scatter_idx=2, gather_idx=1, sp_stream=None):
        super().__init__()
        self.local_attn = local_attention
        self.spg = sequence_process_group
        self.scatter_idx, self.gather_idx = scatter_idx, gather_idx
        self.sp_stream = sp_stream

    def forward(self, query, key, value, *args, **kwargs):
        assert self.scatter_idx == 2 and self.gather_idx == 1, "layout [B, S, H, D] (scatter heads, gather sequence)"
        P = dist.get_world_size(self.spg)
        B = query.shape[0]
        n_q, n_kv = query.shape[2], key.shape[2]
        if n_q % P == 0 and n_kv % P == 0:
            q, k, v = _SeqAllToAll3.apply(self.spg, B, query, key, value)
            ctx = self.local_attn(q, k, v, *args, **kwargs)
            return _SeqAllToAll.apply(self.spg, ctx, self.gather_idx, self.scatter_idx)
        plan = ulysses_head_plan(n_q, n_kv, P)
        me = dist.get_rank(self.spg)

        def go(t, heads):
            y = seq_to_heads(t.reshape(-1, t.shape[2], t.shape[3]), self.spg, B, heads)
            return y.view(B, -1, y.shape[1], y.shape[2])

        q = go(query, [p[0] for p in plan])
        k = go(key, [p[1] for p in plan])
        v = go(value, [p[1] for p in plan])
        ctx = self.local_attn(q, k, v, *args, **kwargs)
        assert ctx.shape[2] == len(plan[me][0])
        o = heads_to_seq(ctx.reshape(-1, ctx.shape[2], ctx.shape[3]), self.spg, B, [len(p[0]) for p in plan])
        return o.view(B, -1, o.shape[1], o.shape[2])


def qkv_head_permutation(n_q, n_kv, P):
    """Index order putting rank r's (q, k, v) heads contiguously: [q_0 k_0 v_0 | q_1 k_1 v_1 | ...]."""
    lq, lkv = n_q // P, n_kv // P
    idx = []
    for r in range(P):
        idx += list(range(r * lq, (r + 1) * lq))
        idx += list(range(n_q + r * lkv, n_q + (r + 1) * lkv))
        idx += list(range(n_q + n_kv + r * lkv, n_q + n_kv + (r + 1) * lkv))
    return idx


def local_heads(n_q, n_kv, group):
    """(local query heads, local kv heads) of this rank under ``ulysses_head_plan``."""
    P = dist.get_world_size(group)
    if n_q % P == 0 and n_kv % P == 0:
        return n_q // P, n_kv // P
    q, kv = ulysses_head_plan(n_q, n_kv, P)[dist.get_rank(group)]
    return len(q), len(kv)


def ulysses_qkv(qkv, n_q, n_kv, group, B):
    """[B*S/P, n_q+2n_kv, D] -> [B*S, nq_r + 2 nkv_r, D] with my heads in q|k|v order (differentiable). Even heads:
    one all-to-all of the fused projection; otherwise the uneven / kv-replicating plan."""
    P = dist.get_world_size(group)
    if n_q % P == 0 and n_kv % P == 0:
        perm = torch.tensor(qkv_head_permutation(n_q, n_kv, P), device=qkv.device)
        return _SeqToHead.apply(qkv.index_select(1, perm), group, B)
    plan = ulysses_head_plan(n_q, n_kv, P)
    send = [q + [n_q + k for k in kv] + [n_q + n_kv + k for k in kv] for q, kv in plan]
    return seq_to_heads(qkv, group, B, send)


def ulysses_out(o, group, B, n_q=None, n_kv=None):
    """[B*S, nq_r, D] -> [B*S/P, n_q, D] (differentiable)."""
    P = dist.get_world_size(group)
    if n_q is None or (n_q % P == 0 and n_kv % P == 0):
        return _HeadToSeq.apply(o, group, B)
    return heads_to_seq(o, group, B, [len(q) for q, _ in ulysses_head_plan(n_q, n_kv, P)])


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
