"""Ring attention (context parallelism) over xGMI point-to-point links.

The reference has NO ring attention / context parallelism (SURVEY.md §2.4 "CP / Ring attention: no",
§5.7 item 5); long context there is Ulysses (sequence/layer.py) + FPDT (sequence/fpdt_layer.py) only.
This is the new strategy planned in SURVEY.md §7.2 (``parallel/ring_attention.py``).

Design (MI355X-first):

* Zigzag (load-balanced causal) layout: the global sequence is cut into ``2P`` chunks of ``c`` tokens;
  rank ``r`` holds chunks ``r`` and ``2P-1-r``. With that layout every ring step does exactly two
  ``c x c`` FlashAttention blocks on every rank (the diagonal step does two causal blocks + one full
  block), so no rank idles on the causal triangle.
* Every block is a dense equal-length launch of the HIP FlashAttention kernel (``attn_block_fwd`` /
  ``attn_block_bwd``); partial results merge in fp32 with their LSE (online softmax).
* K|V of the current source rank travel around the ring in ONE packed buffer per step through
  ``batch_isend_irecv`` (RCCL send/recv on one xGMI link each way), issued BEFORE the step's compute so
  the transfer overlaps the attention blocks. GQA makes the KV message ``2*Hkv/Hq`` the size of Q.
* Backward is the exact blockwise decomposition against the final (o, lse): dq accumulates locally in
  fp32, while the (k, v) of each source rank and its fp32 (dk, dv) accumulator circulate together so
  that after ``P`` hops every rank gets its own dk/dv home. The next hop's k/v are prefetched while the
  current step computes; only the dk/dv hop waits on compute.

On a fully connected 8-GPU xGMI mesh a ring uses one link in / one out per GPU (~153 GB/s) -- Ulysses'
all-to-all uses all 7. Ring attention therefore wins only when heads are too few for Ulysses (P > Hkv) or
is composed with Ulysses (Ulysses inside, ring across); the API takes any process group for that.
"""
import math

import torch
import torch.distributed as tdist

from .. import comm as dist
from ..ops.attention import attn_block_bwd, attn_block_fwd, merge_attn_out


def zigzag_indices(seq_len, sp_size, sp_rank):
    """Global token indices held by ``sp_rank`` in the zigzag layout (chunks r and 2P-1-r)."""
    assert seq_len % (2 * sp_size) == 0, "ring attention needs seq_len divisible by 2 * sp_size"
    c = seq_len // (2 * sp_size)
    a = torch.arange(sp_rank * c, (sp_rank + 1) * c)
    j = 2 * sp_size - 1 - sp_rank
    b = torch.arange(j * c, (j + 1) * c)
    return torch.cat([a, b])


def zigzag_shard(x, sp_size, sp_rank, dim=1):
    """Select this rank's zigzag shard of a full-sequence tensor along ``dim``."""
    idx = zigzag_indices(x.shape[dim], sp_size, sp_rank).to(x.device)
    return x.index_select(dim, idx)


def zigzag_unshard(shards, dim=1):
    """Inverse of :func:`zigzag_shard` given the list of every rank's shard (testing / gathering)."""
    P = len(shards)
    S = shards[0].shape[dim] * P
    out_shape = list(shards[0].shape)
    out_shape[dim] = S
    out = shards[0].new_empty(out_shape)
    for r, s in enumerate(shards):
        idx = zigzag_indices(S, P, r).to(s.device)
        out.index_copy_(dim, idx, s)
    return out


def _blocks(r, j, causal):
    """(q_chunk, k_chunk, causal) blocks for local q chunks {0: chunk r, 1: chunk 2P-1-r} against the k
    chunks {0: chunk j, 1: chunk 2P-1-j} of source rank ``j``."""
    if not causal:
        return [(0, 0, False), (0, 1, False), (1, 0, False), (1, 1, False)]
    if j == r:
        return [(0, 0, True), (1, 0, False), (1, 1, True)]
    if j < r:
        return [(0, 0, False), (1, 0, False)]
    return [(1, 0, False), (1, 1, False)]


class _Ring:
    """Neighbour send/recv over a process group; one batched P2P launch per hop."""

    def __init__(self, group):
        self.group = group
        self.P = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        self.nxt = dist.get_global_rank(group, (self.r + 1) % self.P)
        self.prv = dist.get_global_rank(group, (self.r - 1) % self.P)

    def start(self, bufs):
        recvs = [torch.empty_like(b) for b in bufs]
        ops = []
        for b, rb in zip(bufs, recvs):
            ops.append(tdist.P2POp(tdist.isend, b, self.nxt, self.group))
            ops.append(tdist.P2POp(tdist.irecv, rb, self.prv, self.group))
        return recvs, tdist.batch_isend_irecv(ops)

    @staticmethod
    def wait(pending):
        recvs, reqs = pending
        for q in reqs:
            q.wait()
        return recvs


def _chunk_major(x, B):
    """[B*2c, H, D] (per-sequence zigzag order a|b) -> [2, B*c, H, D] contiguous."""
    T, H, D = x.shape
    c = T // (2 * B)
    return x.view(B, 2, c, H, D).transpose(0, 1).reshape(2, B * c, H, D)


def _token_major(x, B):
    """Inverse of :func:`_chunk_major`."""
    _, Tc, H, D = x.shape
    c = Tc // B
    return x.view(2, B, c, H, D).transpose(0, 1).reshape(B * 2 * c, H, D)


def ring_attn_forward(q, k, v, group, B, causal, scale):
    """q: [2, B*c, Hq, D], k/v: [2, B*c, Hkv, D] (chunk-major). Returns o (q dtype), lse [2, Hq, B*c] fp32."""
    ring = _Ring(group)
    P, r = ring.P, ring.r
    seq = q.shape[1] // B
    o_acc, lse_acc = [None, None], [None, None]
    kv = torch.stack([k, v])  # [2 (k|v), 2 (chunk), B*c, Hkv, D]
    for s in range(P):
        j = (r - s) % P
        pending = ring.start([kv]) if s < P - 1 else None  # next hop overlaps this step's blocks
        for (qi, ki, cz) in _blocks(r, j, causal):
            ob, lb = attn_block_fwd(q[qi], kv[0, ki], kv[1, ki], cz, scale, seq)
            o_acc[qi], lse_acc[qi] = merge_attn_out(o_acc[qi], lse_acc[qi], ob, lb)
        if pending is not None:
            kv = _Ring.wait(pending)[0]
    o = torch.stack([o_acc[0].to(q.dtype), o_acc[1].to(q.dtype)])
    lse = torch.stack([lse_acc[0], lse_acc[1]])
    return o, lse


def ring_attn_backward(q, k, v, o, lse, do, group, B, causal, scale):
    ring = _Ring(group)
    P, r = ring.P, ring.r
    seq = q.shape[1] // B
    dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    kv = torch.stack([k, v])
    dkv = torch.zeros(kv.shape, dtype=torch.float32, device=k.device)
    for s in range(P):
        j = (r - s) % P
        kv_next = ring.start([kv]) if s < P - 1 else None
        for (qi, ki, cz) in _blocks(r, j, causal):
            gq, gk, gv = attn_block_bwd(q[qi], kv[0, ki], kv[1, ki], o[qi], lse[qi], do[qi], cz, scale, seq)
            dq[qi] += gq.float()
            dkv[0, ki] += gk.float()
            dkv[1, ki] += gv.float()
        # dk/dv of source j follow its k/v one hop; after P hops they are back on rank j
        dkv = _Ring.wait(ring.start([dkv]))[0]
        if kv_next is not None:
            kv = _Ring.wait(kv_next)[0]
    return dq.to(q.dtype), dkv[0].to(k.dtype), dkv[1].to(v.dtype)


class _RingAttnFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, k, v, group, B, causal, scale):
        qc, kc, vc = _chunk_major(q, B), _chunk_major(k, B), _chunk_major(v, B)
        o, lse = ring_attn_forward(qc, kc, vc, group, B, causal, scale)
        ctx.save_for_backward(qc, kc, vc, o, lse)
        ctx.args = (group, B, causal, scale)
        return _token_major(o, B)

    @staticmethod
    def backward(ctx, do):
        qc, kc, vc, o, lse = ctx.saved_tensors
        group, B, causal, scale = ctx.args
        doc = _chunk_major(do.contiguous(), B)
        dq, dk, dv = ring_attn_backward(qc, kc, vc, o, lse, doc, group, B, causal, scale)
        return _token_major(dq, B), _token_major(dk, B), _token_major(dv, B), None, None, None, None


def ring_attention(q, k, v, group, causal=True, softmax_scale=None):
    """Context-parallel attention. q: [B, S_local, Hq, D]; k/v: [B, S_local, Hkv, D] in the zigzag layout
    (:func:`zigzag_shard`). Returns o [B, S_local, Hq, D]. ``group`` = the context-parallel process group."""
    B, Sl, Hq, D = q.shape
    assert Sl % 2 == 0, "zigzag layout holds two chunks per rank"
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    q3 = q.reshape(B * Sl, Hq, D)
    k3 = k.reshape(B * Sl, k.shape[2], D)
    v3 = v.reshape(B * Sl, v.shape[2], D)
    o = _RingAttnFn.apply(q3, k3, v3, group, B, bool(causal), float(scale))
    return o.view(B, Sl, Hq, D)


class RingAttention(torch.nn.Module):
    """Module wrapper with ``DistributedAttention``'s call signature (q, k, v as [B, S/P, H, D], zigzag)."""

    def __init__(self, cp_process_group, causal=True, softmax_scale=None):
        super().__init__()
        self.group = cp_process_group
        self.causal = causal
        self.scale = softmax_scale

    def forward(self, query, key, value, *args, **kwargs):
        return ring_attention(query, key, value, self.group, causal=self.causal, softmax_scale=self.scale)
