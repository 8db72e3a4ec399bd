"""FPDT (Ulysses-Offload): chunked Ulysses attention with host-offloaded chunks, chunked FFN and logits loss.

Reference parity: sequence/fpdt_layer.py -- ``FPDT_InputConstruct`` :79-131 (load-balanced chunk layout),
``_FPDTGPUAttentionImpl_`` :134-459 / ``_FPDTGPUOffloadingAttentionImpl_`` :510-968 (per-chunk QKV GEMM,
all-to-all, flash-attn over all previous KV chunks with an online-softmax merge ``update_out_and_lse``
:40-76, blockwise backward), ``SequenceChunk`` :462-508 (host offload), ``FPDT_Attention`` :971-1041,
``FPDT_FFN`` :1056-1134 and ``FPDT_LogitsLoss`` :1137-1225.

MI355X design:

* Token layout: rank r holds global chunks r, r+P, r+2P, ... so that after the all-to-all of local chunk i
  every rank sees the CONTIGUOUS global segment i (P*chunk tokens) for its H/P heads. Causal attention is
  then "segment i attends fully to segments < i and causally to itself" -- every block is a dense
  equal-length FlashAttention launch (the HIP kernel, no padding / masks).
* One all-to-all per chunk moves the fused q|k|v heads (weight rows are permuted once per call so each
  rank's q|k|v heads are contiguous, as in parallel/ulysses.py), RoPE runs in place with a position
  offset, and partial results are merged in fp32 with their LSE.
* Offload: the post-RoPE q/k/v, merged o and lse of every segment go to PINNED host buffers on a side
  copy stream (event-ordered); backward streams them back one KV segment ahead of use (double buffering)
  so only O(2 segments) of attention state lives in HBM. On a 288 GB MI355X this is for the 1M+ token
  regime; below that, ``offload=False`` keeps everything resident.
* Backward loops KV segments j (outer) and query segments i >= j (inner) with the exact blockwise
  decomposition (global o / lse per query segment, ``attn_block_bwd``); dk_j / dv_j finish after their
  inner loop and dq_j after iteration j, so the dqkv of segment j is all-to-all'ed back and folded into
  dx / dW immediately.
"""
import math

import torch

from .. import comm as dist
from ..ops.attention import attn_block_bwd, attn_block_fwd, merge_attn_out
from ..ops.cross_entropy import _addmm_f32_
from ..ops.rope import rope_
from .ulysses import head_to_seq, qkv_head_permutation, seq_to_head


class FPDTInputConstruct:
    """Reorders a global batch into this rank's load-balanced FPDT layout (reference :79-131)."""

    def __init__(self, tokens, labels, loss_mask, attention_mask, position_ids, chunk_size, sp_size, sp_rank):
        S = tokens.shape[1]
        assert S % sp_size == 0 and S % chunk_size == 0, "sequence must divide sp_size and the FPDT chunk size"
        self.num_chunk_per_gpu = S // chunk_size
        self.local_seq_len = S // sp_size
        assert self.local_seq_len % self.num_chunk_per_gpu == 0
        self.chunk_size = self.local_seq_len // self.num_chunk_per_gpu
        self.tokens, self.labels, self.loss_mask = tokens, labels, loss_mask
        self.attention_mask, self.position_ids = attention_mask, position_ids
        self.sp_size, self.sp_rank = sp_size, sp_rank

    def indices(self):
        cs, nc, P = self.chunk_size, self.num_chunk_per_gpu, self.sp_size
        chunks = [i * P + self.sp_rank for i in range(nc)]  # global chunk ids held by this rank, in order
        return torch.cat([torch.arange(c * cs, (c + 1) * cs) for c in chunks])

    def generate(self):
        idx = self.indices().to(self.tokens.device)
        sel = (lambda t: t[:, idx] if t is not None else None)
        return (sel(self.tokens), sel(self.labels), sel(self.loss_mask), self.attention_mask,
                sel(self.position_ids))


def fpdt_layout_indices(seq_len, chunk_size, sp_size, sp_rank):
    """Global token indices held by ``sp_rank`` (``chunk_size`` = global FPDT chunk = P * local chunk)."""
    ic = FPDTInputConstruct(torch.zeros(1, seq_len, dtype=torch.long), None, None, None, None, chunk_size, sp_size,
                            sp_rank)
    return ic.indices()


class _HostChunks:
    """Segment store: device tensors, or pinned host copies written/read on a side HIP stream."""

    def __init__(self, offload, device):
        self.offload = bool(offload) and device.type == "cuda"
        self.stream = torch.cuda.Stream(device, priority=-1) if self.offload else None
        self.host, self.ready, self.dev = {}, {}, {}

    def put(self, key, t):
        if not self.offload:
            self.dev[key] = t
            return
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        cur = torch.cuda.current_stream(t.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            h.copy_(t, non_blocking=True)
            t.record_stream(self.stream)
        self.host[key] = h

    def prefetch(self, key, device):
        if not self.offload or key in self.ready or key not in self.host:
            return
        with torch.cuda.stream(self.stream):
            d = torch.empty(self.host[key].shape, dtype=self.host[key].dtype, device=device)
            d.copy_(self.host[key], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.ready[key] = (d, ev)

    def get(self, key, device=None):
        if not self.offload:
            return self.dev[key]
        self.prefetch(key, device)
        d, ev = self.ready.pop(key)
        torch.cuda.current_stream(d.device).wait_event(ev)
        d.record_stream(torch.cuda.current_stream(d.device))
        return d

    def drop(self, key):
        self.dev.pop(key, None)
        self.host.pop(key, None)
        self.ready.pop(key, None)


def _permuted_weight(w, b, n_q, n_kv, D, P):
    perm = torch.tensor(qkv_head_permutation(n_q, n_kv, P), device=w.device)
    wp = w.view(n_q + 2 * n_kv, D, -1).index_select(0, perm).reshape(w.shape)
    bp = None if b is None else b.view(n_q + 2 * n_kv, D).index_select(0, perm).reshape(-1)
    return wp, bp, perm


class _FPDTAttnFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, w, b, cos, sin, n_q, n_kv, D, group, B, num_chunks, offload, scale, keep=True):
        """x [B*Sl, H] (FPDT layout) -> attention output [B*Sl, n_q*D] (before the output projection).

        ``keep`` False (a no-grad forward, e.g. the first pass of a checkpointed block): nothing goes to the
        segment store -- no backward will read it -- and the previous segments' K/V stay on the device (GQA: 2 GiB
        at 512k tokens), so the forward moves no bytes over PCIe. Inside a checkpointed block with the attention
        stash (``ops.attention.AttnStash``), "record" keeps every segment's merged (o, lse) and "replay" -- the
        backward's recompute -- takes them back instead of re-running the segment-pair attention (at 512k tokens
        about a sixth of the step)."""
        from ..ops.attention import AttnStash
        mode = AttnStash.mode
        P = dist.get_world_size(group) if group is not None else 1
        T, H = x.shape
        Sl = T // B
        cs = Sl // num_chunks
        assert cs * num_chunks == Sl, f"local sequence {Sl} not divisible into {num_chunks} FPDT chunks"
        nql, nkvl = n_q // P, n_kv // P
        L = P * cs  # global segment length
        wp, bp, perm = _permuted_weight(w, b, n_q, n_kv, D, P)
        xv = x.view(B, Sl, H)
        store = _HostChunks(offload and keep, x.device)
        out = torch.empty(B, Sl, n_q * D, device=x.device, dtype=x.dtype)
        ks, vs = [], []  # previous segments' K/V (device-resident unless offloading)
        for i in range(num_chunks):
            xi = xv[:, i * cs:(i + 1) * cs].reshape(B * cs, H)
            qkv = torch.nn.functional.linear(xi, wp, bp).view(B * cs, n_q + 2 * n_kv, D)
            full = seq_to_head(qkv, group, B) if P > 1 else qkv  # [B*L, nql+2nkvl, D]
            rope_(full, cos, sin, nql + nkvl, seq_len=L, pos_offset=i * L)
            q = full[:, :nql].contiguous()
            k = full[:, nql:nql + nkvl].contiguous()
            v = full[:, nql + nkvl:].contiguous()
            if mode == "replay":
                o, lse = AttnStash.items.pop(0)
                assert o.shape == q.shape and lse.shape == (nql, q.shape[0]), "FPDT attention stash out of order"
            else:
                o, lse = None, None
                for j in range(i):
                    if store.offload:
                        if j + 1 < i:
                            store.prefetch(("k", j + 1), x.device)
                            store.prefetch(("v", j + 1), x.device)
                        kj, vj = store.get(("k", j), x.device), store.get(("v", j), x.device)
                    else:
                        kj, vj = ks[j], vs[j]
                    ob, lb = attn_block_fwd(q, kj, vj, False, scale, L)
                    o, lse = merge_attn_out(o, lse, ob, lb)
                ob, lb = attn_block_fwd(q, k, v, True, scale, L)
                o, lse = merge_attn_out(o, lse, ob, lb)
                if not store.offload:
                    ks.append(k)
                    vs.append(v)
                o = o.to(x.dtype)
                if mode == "record":
                    AttnStash.items.append((o, lse))
            oo = head_to_seq(o, group, B) if P > 1 else o  # [B*cs, n_q, D]
            out[:, i * cs:(i + 1) * cs] = oo.view(B, cs, n_q * D)
            if keep:
                for key, t in (("q", q), ("k", k), ("v", v), ("o", o), ("lse", lse)):
                    store.put((key, i), t)
        ctx.save_for_backward(x, wp, bp)
        ctx.store, ctx.perm, ctx.has_b = store, perm, b is not None
        ctx.meta = (n_q, n_kv, D, group, B, num_chunks, scale, P, cs, L)
        ctx.cos, ctx.sin = cos, sin
        return out.view(T, n_q * D)

    @staticmethod
    def backward(ctx, dout):
        x, wp, bp = ctx.saved_tensors
        n_q, n_kv, D, group, B, nc, scale, P, cs, L = ctx.meta
        store, dev = ctx.store, x.device
        nql, nkvl = n_q // P, n_kv // P
        T, H = x.shape
        Sl = T // B
        dov = dout.contiguous().view(B, Sl, n_q, D)
        # do of every query segment, in head layout (kept alongside q/o/lse in the store)
        for i in range(nc):
            di = dov[:, i * cs:(i + 1) * cs].reshape(B * cs, n_q, D)
            store.put(("do", i), seq_to_head(di, group, B) if P > 1 else di.contiguous())
        dq_acc = [None] * nc
        dx = torch.empty_like(x).view(B, Sl, H)
        dwp = torch.zeros(wp.shape, device=dev, dtype=torch.float32)
        dbp = torch.zeros(wp.shape[0], device=dev, dtype=torch.float32) if ctx.has_b else None
        xv = x.view(B, Sl, H)
        for j in range(nc):
            k, v = store.get(("k", j), dev), store.get(("v", j), dev)
            dk = torch.zeros(k.shape, device=dev, dtype=torch.float32)
            dv = torch.zeros(v.shape, device=dev, dtype=torch.float32)
            for i in range(j, nc):
                q, o, lse, do = (store.get((n, i), dev) for n in ("q", "o", "lse", "do"))
                nxt = [(n, i + 1) for n in ("q", "o", "lse", "do")] if i + 1 < nc else \
                    [(n, j + 1) for n in ("k", "v", "q", "o", "lse", "do")] if j + 1 < nc else []
                for key in nxt:
                    store.prefetch(key, dev)
                gq, gk, gv = attn_block_bwd(q, k, v, o, lse, do, i == j, scale, L)
                dk += gk
                dv += gv
                dq_acc[i] = gq.float() if dq_acc[i] is None else dq_acc[i].add_(gq)
            # segment j is complete: inverse RoPE, all-to-all back, fold into dx / dW
            dqkv = torch.cat([dq_acc[j], dk, dv], dim=1).to(x.dtype)
            dq_acc[j] = None
            rope_(dqkv, ctx.cos, ctx.sin, nql + nkvl, seq_len=L, pos_offset=j * L, sign=-1.0)
            loc = head_to_seq(dqkv, group, B) if P > 1 else dqkv  # [B*cs, NH, D] permuted head order
            g2 = loc.reshape(B * cs, -1)
            xj = xv[:, j * cs:(j + 1) * cs].reshape(B * cs, H)
            dx[:, j * cs:(j + 1) * cs] = (g2 @ wp).view(B, cs, H)
            _addmm_f32_(dwp, g2.t(), xj)  # bf16 GEMM, fp32 accumulator folded in (no fp32 operand copies)
            if dbp is not None:
                dbp += g2.float().sum(0)
            for n in ("q", "k", "v", "o", "lse", "do"):  # later kv segments only touch query segments > j
                store.drop((n, j))
        inv = torch.empty_like(ctx.perm)
        inv[ctx.perm] = torch.arange(ctx.perm.numel(), device=dev)
        dw = dwp.view(n_q + 2 * n_kv, D, H).index_select(0, inv).reshape(wp.shape).to(wp.dtype)
        db = None if dbp is None else dbp.view(n_q + 2 * n_kv, D).index_select(0, inv).reshape(-1).to(bp.dtype)
        ctx.store = None
        return dx.view(T, H), dw, db, None, None, None, None, None, None, None, None, None, None, None


def fpdt_attention(x, qkv_weight, qkv_bias, cos, sin, n_q, n_kv, head_dim, group, batch, num_chunks,
                   offload=False, softmax_scale=None):
    """Causal FPDT attention core: [B*Sl, H] (FPDT layout) -> [B*Sl, n_q*head_dim]."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(head_dim)
    keep = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (x, qkv_weight, qkv_bias))
    return _FPDTAttnFn.apply(x, qkv_weight, qkv_bias, cos, sin, n_q, n_kv, head_dim, group, batch, num_chunks,
                             offload, scale, keep)


class FPDT_Attention(torch.nn.Module):
    """Module form (reference :971-1041): fused QKV weight/bias + output projection around fpdt_attention."""

    def __init__(self, config, first_weight, first_bias, second_weight, second_bias, sequence_process_group,
                 gather_idx=0, scatter_idx=2, return_bias=True, chunk_size=65536, enable_offloading=True):
        super().__init__()
        self.spg = sequence_process_group
        self.n_q = config.num_attention_heads
        self.n_kv = getattr(config, "num_key_value_heads", self.n_q)
        self.d = getattr(config, "head_dim", None) or config.hidden_size // self.n_q
        self.qkv_weight, self.qkv_bias = first_weight, first_bias
        self.out_weight, self.out_bias = second_weight, second_bias
        self.return_bias = return_bias
        self.chunk_size = chunk_size
        self.offload = enable_offloading

    def forward(self, hidden, cos, sin, batch=1, cpu_offloading=True):
        P = dist.get_world_size(self.spg) if self.spg is not None else 1
        T = hidden.shape[0]
        nc = max(1, (T // batch) * P // self.chunk_size)
        o = fpdt_attention(hidden, self.qkv_weight, self.qkv_bias, cos, sin, self.n_q, self.n_kv, self.d, self.spg,
                           batch, nc, offload=self.offload and cpu_offloading)
        out = torch.nn.functional.linear(o, self.out_weight)
        if self.return_bias:
            return out, self.out_bias
        return (out + self.out_bias if self.out_bias is not None else out), None


class _ChunkedFn(torch.autograd.Function):
    """Sequence-chunked recompute: fn(x_chunk, *params) is evaluated chunk by chunk with no saved activations
    and re-run per chunk in backward (FPDT_FFN :1056-1134 generalised to any token-wise block)."""

    @staticmethod
    def forward(ctx, fn, num_chunks, x, *params):
        ctx.fn, ctx.nc = fn, num_chunks
        ctx.save_for_backward(x, *params)
        with torch.no_grad():
            return torch.cat([fn(c, *params) for c in x.chunk(num_chunks, 0)], 0)

    @staticmethod
    def backward(ctx, g):
        x, *params = ctx.saved_tensors
        dx = torch.empty_like(x)
        grads = [None if not p.requires_grad else torch.zeros_like(p, dtype=torch.float32) for p in params]
        off = 0
        for c, gc in zip(x.chunk(ctx.nc, 0), g.chunk(ctx.nc, 0)):
            with torch.enable_grad():
                cc = c.detach().requires_grad_(True)
                ps = [p.detach().requires_grad_(p.requires_grad) for p in params]
                y = ctx.fn(cc, *ps)
                need = [cc] + [p for p in ps if p.requires_grad]
                gs = torch.autograd.grad(y, need, gc)
            dx[off:off + c.shape[0]] = gs[0]
            off += c.shape[0]
            it = iter(gs[1:])
            for k, p in enumerate(ps):
                if p.requires_grad:
                    grads[k] += next(it).float()
        return (None, None, dx, *[None if gr is None else gr.to(p.dtype) for gr, p in zip(grads, params)])


def chunked_apply(fn, x, *params, num_chunks=1):
    """Apply the token-wise ``fn(x, *params)`` in ``num_chunks`` sequence chunks with per-chunk recompute."""
    if num_chunks <= 1:
        return fn(x, *params)
    return _ChunkedFn.apply(fn, num_chunks, x, *params)


def _gated_ffn(x, w_up, w_down, act="silu"):
    from ..ops.activations import glu
    return torch.nn.functional.linear(glu(torch.nn.functional.linear(x, w_up), act), w_down)


def _bias_gelu_ffn(x, w1, b1, w2, b2):
    h = torch.nn.functional.gelu(torch.nn.functional.linear(x, w1, b1), approximate="tanh")
    return torch.nn.functional.linear(h, w2, b2)


def FPDT_FFN(x, w1, b1, w2, b2, add_bias=True, chunk_size=None):
    """Reference-signature chunked GELU MLP (:1056): returns (out, bias-or-None)."""
    nc = max(1, x.shape[0] // chunk_size) if chunk_size else 1
    if add_bias:
        return chunked_apply(_bias_gelu_ffn, x, w1, b1, w2, b2, num_chunks=nc), None
    return chunked_apply(lambda t, a, c, d: _bias_gelu_ffn(t, a, c, d, None), x, w1, b1, w2, num_chunks=nc), b2


def fpdt_gated_ffn(x, w_up, w_down, num_chunks, act="silu"):
    return chunked_apply(lambda t, a, b: _gated_ffn(t, a, b, act), x, w_up, w_down, num_chunks=num_chunks)


class _LogitsLossFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, h, weight, labels, num_chunks):
        T = h.shape[0]
        loss = torch.empty(T, device=h.device, dtype=torch.float32)
        with torch.no_grad():
            for idx in torch.arange(T, device=h.device).chunk(num_chunks):
                lg = torch.nn.functional.linear(h[idx], weight).float()
                loss[idx] = torch.nn.functional.cross_entropy(lg, labels[idx], reduction="none", ignore_index=-100)
        ctx.save_for_backward(h, weight, labels)
        ctx.nc = num_chunks
        return loss

    @staticmethod
    def backward(ctx, g):
        h, weight, labels = ctx.saved_tensors
        dh = torch.empty_like(h)
        dw = torch.zeros(weight.shape, device=h.device, dtype=torch.float32)
        for idx in torch.arange(h.shape[0], device=h.device).chunk(ctx.nc):
            lg = torch.nn.functional.linear(h[idx], weight).float()
            p = torch.softmax(lg, -1)
            lab = labels[idx]
            valid = lab != -100
            p[torch.arange(p.shape[0], device=p.device)[valid], lab[valid]] -= 1.0
            p *= (g[idx] * valid)[:, None]
            if h.is_cuda and h.dtype != torch.float32:
                # bf16 GEMMs with fp32 accumulation: no fp32 copy of the [V, H] LM-head weight per chunk
                pl = p.to(h.dtype)
                dh[idx] = pl @ weight
                _addmm_f32_(dw, pl.t(), h[idx])
            else:
                dh[idx] = (p @ weight.float()).to(h.dtype)
                dw.addmm_(p.t(), h[idx].float())
        return dh, dw.to(weight.dtype), None, None


def FPDT_LogitsLoss(h, labels, weight, sp_group=None, num_chunks=1):
    """Per-token CE losses of this rank's tokens (chunked logits, recomputed in backward), all-gathered over
    the sequence-parallel group: returns [P * T_local] fp32 (reference :1137-1225)."""
    loss = _LogitsLossFn.apply(h, weight, labels, num_chunks)
    if sp_group is None or dist.get_world_size(sp_group) == 1:
        return loss
    from .ulysses import _a2a  # noqa: F401  (keeps the group import local)
    return _AllGatherLoss.apply(loss, sp_group)


class _AllGatherLoss(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        P = dist.get_world_size(group)
        out = torch.empty(P * x.numel(), device=x.device, dtype=x.dtype)
        dist.all_gather_into_tensor(out, x.contiguous(), group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        r = dist.get_rank(ctx.group)
        n = g.numel() // dist.get_world_size(ctx.group)
        return g[r * n:(r + 1) * n].contiguous(), None


def enable_fpdt(model, group, chunk_size, offload=True, ffn_chunks=0):
    """Turn every LlamaAttention into FPDT attention (``chunk_size`` = global tokens per segment). Inputs must
    be in the :class:`FPDTInputConstruct` layout. ``ffn_chunks`` > 1 also chunks the MLPs."""
    from ..models.llama import LlamaAttention, LlamaMLP
    P = dist.get_world_size(group) if group is not None else 1
    n = 0
    for m in model.modules():
        if isinstance(m, LlamaAttention):
            m.fpdt = dict(group=group, chunk_size=chunk_size, offload=offload)
            n += 1
        if isinstance(m, LlamaMLP) and ffn_chunks > 1:
            m.fpdt_chunks = ffn_chunks
        if hasattr(m, "rope") and hasattr(m, "layers"):
            m._hds_sp_size = P
    return n
