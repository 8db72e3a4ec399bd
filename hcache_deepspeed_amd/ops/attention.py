"""FlashAttention (causal / sliding window / full, GQA, varlen) with HIP forward+backward.

Reference parity: replaces ``BlockedFlashAttn`` (inference/v2/kernels/ragged_ops/blocked_flash,
a prebuilt NVIDIA-only library), the ``flash_attn`` dependency of FPDT
(sequence/fpdt_layer.py:234-254) and the training attention that HF models run unfused.

Head dims: every multiple of 16 up to 256 that the kernel library instantiates (32 ... 256, see
``head_dim_supported``) runs the HIP kernels; bf16 only. A right-padded batch with a key-padding mask runs
the same kernels with per-sequence lengths (``seq_lens``).

Two entry points:

* :func:`flash_attn` -- q/k/v as ``[B, S, H, D]`` or varlen ``[T, H, D]`` + ``cu_seqlens``;
  returns ``o`` (and optionally the fp32 LSE used by FPDT / ring-attention merges).
* :func:`qkv_attention` -- the training fast path: consumes the fused QKV GEMM output
  ``[T, Hq + 2*Hkv, D]``, applies RoPE in place, runs attention on strided views of the same
  buffer, and in backward writes dq/dk/dv straight into one ``[T, Hq + 2*Hkv, D]`` gradient that
  the QKV GEMM's backward consumes. No split / transpose / cat copies exist on either pass.
"""
import math

import torch

from . import native
from .rope import rope_
from ..offload import act_plan as _ap

_HEAD_DIMS_NATIVE = (32, 48, 64, 80, 96, 112, 128, 160, 192, 256)  # mirrors HDS_ATTN_DIMS in flash_attn.hip


def head_dim_supported(d):
    """True when the HIP attention kernels are instantiated for head_dim ``d``."""
    if torch.cuda.is_available():
        return bool(native.kernels().hds_attn_head_dim_supported(int(d)))
    return d in _HEAD_DIMS_NATIVE


def _strides8(*ts):
    vals = []
    for t in ts:
        vals.append(0 if t is None else t.stride(0))
    while len(vals) < 8:
        vals.append(0)
    return torch.tensor(vals, dtype=torch.int64)


def _check_tok_layout(t, name):
    assert t.dim() == 3 and t.stride(2) == 1 and t.stride(1) == t.shape[2], \
        f"{name}: expected [T, H, D] with contiguous head blocks, got shape {tuple(t.shape)} strides {t.stride()}"


def _cu_info(cu_seqlens, T, seq_len):
    if cu_seqlens is None:
        B = T // seq_len
        return None, B, seq_len, seq_len
    cu = cu_seqlens.to(torch.int32).contiguous()
    lens = (cu[1:] - cu[:-1])
    return cu, cu.numel() - 1, 0, int(lens.max().item()) if lens.numel() else 0


def _ref_attention(q, k, v, causal, scale, cu_seqlens, seq_len, window):
    """fp32 torch reference on [T, H, D] tensors; returns o (q.dtype) and lse [Hq, T] fp32."""
    T, Hq, D = q.shape
    Hkv = k.shape[1]
    G = Hq // Hkv
    if cu_seqlens is None:
        bounds = [(i * seq_len, (i + 1) * seq_len) for i in range(T // seq_len)]
    else:
        c = cu_seqlens.tolist()
        bounds = list(zip(c[:-1], c[1:]))
    o = torch.empty(T, Hq, D, dtype=torch.float32, device=q.device)
    lse = torch.empty(Hq, T, dtype=torch.float32, device=q.device)
    for (s, e) in bounds:
        L = e - s
        if L == 0:
            continue
        qs = q[s:e].float().transpose(0, 1)  # [Hq, L, D]
        ks = k[s:e].float().transpose(0, 1).repeat_interleave(G, 0)
        vs = v[s:e].float().transpose(0, 1).repeat_interleave(G, 0)
        sc = torch.matmul(qs, ks.transpose(1, 2)) * scale
        i = torch.arange(L, device=q.device)
        mask = torch.zeros(L, L, dtype=torch.bool, device=q.device)
        if causal:
            mask |= i[None, :] > i[:, None]
        if window and window > 0:
            mask |= i[None, :] <= i[:, None] - window
        sc = sc.masked_fill(mask, float("-inf"))
        lse[:, s:e] = torch.logsumexp(sc, dim=-1)
        o[s:e] = torch.matmul(torch.softmax(sc, dim=-1), vs).transpose(0, 1)
    return o.to(q.dtype), lse


def _native_fwd(q, k, v, o, lse, causal, scale, cu, B, seq_len, max_len, window, seq_lens=None):
    T, Hq, D = q.shape
    strides = _strides8(q, k, v, o)
    native.check(
        native.kernels().hds_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                                      strides.data_ptr(), native.ptr(cu), native.ptr(seq_lens), B, seq_len, max_len,
                                      T, Hq, k.shape[1], D, float(scale), int(causal), int(window), native.stream()),
        "attn_fwd")


def _native_bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale, cu, B, seq_len, max_len, window, seq_lens=None):
    T, Hq, D = q.shape
    delta = torch.empty(2, Hq, T, device=q.device, dtype=torch.float32)  # rowsum(dO * O), lse * log2(e)
    strides = _strides8(q, k, v, o, do, dq, dk, dv)
    native.check(
        native.kernels().hds_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                                      do.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), delta.data_ptr(),
                                      strides.data_ptr(), native.ptr(cu), native.ptr(seq_lens), B, seq_len, max_len,
                                      T, Hq, k.shape[1], D, float(scale), int(causal), int(window), native.stream()),
        "attn_bwd")


def _ref_bwd(q, k, v, do, causal, scale, cu_seqlens, seq_len, window):
    with torch.enable_grad():
        qf = q.detach().float().requires_grad_(True)
        kf = k.detach().float().requires_grad_(True)
        vf = v.detach().float().requires_grad_(True)
        o, _ = _ref_attention_f32(qf, kf, vf, causal, scale, cu_seqlens, seq_len, window)
        dq, dk, dv = torch.autograd.grad(o, (qf, kf, vf), do.float())
    return dq, dk, dv


def _ref_attention_f32(q, k, v, causal, scale, cu_seqlens, seq_len, window):
    # differentiable fp32 variant of _ref_attention
    T, Hq, D = q.shape
    G = Hq // k.shape[1]
    if cu_seqlens is None:
        bounds = [(i * seq_len, (i + 1) * seq_len) for i in range(T // seq_len)]
    else:
        c = cu_seqlens.tolist()
        bounds = list(zip(c[:-1], c[1:]))
    outs = []
    for (s, e) in bounds:
        L = e - s
        qs = q[s:e].transpose(0, 1)
        ks = k[s:e].transpose(0, 1).repeat_interleave(G, 0)
        vs = v[s:e].transpose(0, 1).repeat_interleave(G, 0)
        sc = torch.matmul(qs, ks.transpose(1, 2)) * scale
        i = torch.arange(L, device=q.device)
        mask = torch.zeros(L, L, dtype=torch.bool, device=q.device)
        if causal:
            mask |= i[None, :] > i[:, None]
        if window and window > 0:
            mask |= i[None, :] <= i[:, None] - window
        sc = sc.masked_fill(mask, float("-inf"))
        outs.append(torch.matmul(torch.softmax(sc, -1), vs).transpose(0, 1))
    return torch.cat(outs, 0), None


def native_supported(q):
    """bf16 on the GPU with an instantiated head dim -> HIP kernels. A bf16 GPU tensor with any other head dim is
    an error (no silent fp32 fallback on the device); fp16/fp32 inputs use the fp32 reference."""
    if not (native.use_native(q) and q.dtype == torch.bfloat16):
        return False
    if not head_dim_supported(q.shape[-1]):
        raise NotImplementedError(f"HIP attention: head_dim {q.shape[-1]} is not instantiated "
                                  f"(supported: multiples of 16 up to 256)")
    return True


def _padded_ref(q, k, v, causal, scale, seq_len, window, seq_lens):
    """Reference for a right-padded batch: each sequence's first seq_lens[b] rows; padded outputs are zero."""
    lens = seq_lens.tolist()
    o = torch.zeros(q.shape, dtype=q.dtype, device=q.device)
    lse = torch.full((q.shape[1], q.shape[0]), float("-inf"), dtype=torch.float32, device=q.device)
    for b, L in enumerate(lens):
        s = b * seq_len
        if L > 0:
            ob, lb = _ref_attention(q[s:s + L], k[s:s + L], v[s:s + L], causal, scale, None, L, window)
            o[s:s + L] = ob
            lse[:, s:s + L] = lb
    return o, lse


class _FlashAttnFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, cu_seqlens, seq_len, window, return_lse, seq_lens):
        T, Hq, D = q.shape
        cu, B, sl, max_len = _cu_info(cu_seqlens, T, seq_len)
        sls = None if seq_lens is None else seq_lens.to(device=q.device, dtype=torch.int32).contiguous()
        if native_supported(q):
            alloc = torch.zeros if sls is not None else torch.empty  # padded rows are never written
            o = alloc(T, Hq, D, device=q.device, dtype=q.dtype)
            lse = torch.empty(Hq, T, device=q.device, dtype=torch.float32)
            _native_fwd(q, k, v, o, lse, causal, scale, cu, B, sl, max_len, window, sls)
        elif sls is not None:
            o, lse = _padded_ref(q, k, v, causal, scale, seq_len, window, sls)
        else:
            o, lse = _ref_attention(q, k, v, causal, scale, cu_seqlens, seq_len, window)
        ctx.save_for_backward(q, k, v, o, lse, cu_seqlens, sls)
        ctx.args = (causal, scale, seq_len, window)
        ctx.mark_non_differentiable(lse)
        return o, lse

    @staticmethod
    def backward(ctx, do, dlse):
        q, k, v, o, lse, cu_seqlens, sls = ctx.saved_tensors
        causal, scale, seq_len, window = ctx.args
        T = q.shape[0]
        cu, B, sl, max_len = _cu_info(cu_seqlens, T, seq_len)
        if native_supported(q):
            alloc = torch.zeros if sls is not None else torch.empty
            dq = alloc(q.shape, device=q.device, dtype=q.dtype)
            dk = alloc(k.shape, device=k.device, dtype=k.dtype)
            dv = alloc(v.shape, device=v.device, dtype=v.dtype)
            _native_bwd(q, k, v, o, lse, do.contiguous(), dq, dk, dv, causal, scale, cu, B, sl, max_len, window, sls)
        elif sls is not None:
            with torch.enable_grad():
                qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
                of, _ = _padded_ref(qf, kf, vf, causal, scale, seq_len, window, sls)
                dq, dk, dv = torch.autograd.grad(of, (qf, kf, vf), do.float())
            dq, dk, dv = dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)
        else:
            dq, dk, dv = _ref_bwd(q, k, v, do, causal, scale, cu_seqlens, seq_len, window)
            dq, dk, dv = dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype)
        return dq, dk, dv, None, None, None, None, None, None, None


def _count_attn_flops(T, H, D, seq_len, causal, cu_seqlens):
    """Report QK^T + PV flops to a running FlopsProfiler (the HIP kernel is invisible to aten dispatch)."""
    from ..profiling import counters
    if not counters.active():
        return
    if cu_seqlens is not None:
        lens = (cu_seqlens[1:] - cu_seqlens[:-1]).tolist()
    else:
        lens = [seq_len] * (T // max(1, seq_len))
    pairs = sum(L * (L + 1) / 2 if causal else L * L for L in lens)
    counters.add(4 * pairs * H * D, 2 * pairs * H * D, "flash_attn")


def flash_attn(q, k, v, causal=True, softmax_scale=None, cu_seqlens=None, window=0, return_lse=False, seq_lens=None):
    """q: [B, S, Hq, D] or [T, Hq, D] (+cu_seqlens); k/v: [.., Hkv, D]. Returns o like q (and lse [Hq, T]).

    seq_lens: optional int [B] valid lengths of a right-padded [B, S] batch (a key-padding mask); outputs and
    gradients of padded rows are zero."""
    batched = q.dim() == 4
    if batched:
        B, S = q.shape[:2]
        q3, k3, v3 = (t.reshape(B * S, t.shape[2], t.shape[3]) for t in (q, k, v))
        seq_len = S
    else:
        q3, k3, v3 = q, k, v
        seq_len = q.shape[0]
    for t, n in ((q3, "q"), (k3, "k"), (v3, "v")):
        _check_tok_layout(t, n)
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    _count_attn_flops(q3.shape[0], q3.shape[1], q3.shape[2], seq_len, causal, cu_seqlens)
    o, lse = _FlashAttnFn.apply(q3, k3, v3, bool(causal), float(scale), cu_seqlens, int(seq_len), int(window or 0),
                                return_lse, seq_lens)
    if batched:
        o = o.view(q.shape)
    return (o, lse) if return_lse else o


class AttnStash:
    """Attention outputs carried from a checkpointed forward to its recompute (FlashAttention is the costliest part of
    recomputing a block, and its output + LSE are a small part of the block's bytes). ``record``: every attention call
    appends its (o, lse); ``replay``: every attention call takes the next stored pair instead of running the forward
    kernel -- the recompute then re-runs only the projections, norms and MLP
    (runtime/activation_checkpointing/checkpointing.checkpoint_saved_inputs(stash_attention=True))."""
    mode = None  # None | "record" | "replay"
    items = None

    @classmethod
    def active(cls):
        return cls.mode is not None


def _stash_take(T, n_q, D, dtype, device):
    o, lse = AttnStash.items.pop(0)
    assert o.shape[0] == T and o.numel() == T * n_q * D and o.dtype == dtype, "attention stash out of order"
    return o.view(T, n_q, D), lse


def _qkv_recipe(proj, NH, D, n_rot, cos, sin, seq_len, pos_ids):
    """The packed qkv tensor attention saved: the projection's recipe, then RoPE in place (as in forward)."""

    def run(*args):
        y = proj(*args)
        if cos is not None:
            rope_(y.view(-1, NH, D), cos, sin, n_rot, seq_len=seq_len, pos_ids=pos_ids)
        return y

    return run


class _QKVAttnFn(torch.autograd.Function):
    """RoPE(q,k) + attention on the packed QKV GEMM output; see module docstring."""

    @staticmethod
    def forward(ctx, qkv, n_q, n_kv, cos, sin, seq_len, causal, scale, cu_seqlens, pos_ids, window):
        T, NH, D = qkv.shape
        tagged = _ap.lookup(qkv) if _ap.tracking() else None
        if cos is not None:
            rope_(qkv, cos, sin, n_q + n_kv, seq_len=seq_len, pos_ids=pos_ids)  # in place on the GEMM output
        q = qkv[:, :n_q]
        k = qkv[:, n_q:n_q + n_kv]
        v = qkv[:, n_q + n_kv:]
        cu, B, sl, max_len = _cu_info(cu_seqlens, T, seq_len)
        if AttnStash.mode == "replay":
            o, lse = _stash_take(T, n_q, D, qkv.dtype, qkv.device)
        elif native_supported(qkv):
            o = torch.empty(T, n_q, D, device=qkv.device, dtype=qkv.dtype)
            lse = torch.empty(n_q, T, device=qkv.device, dtype=torch.float32)
            _native_fwd(q, k, v, o, lse, causal, scale, cu, B, sl, max_len, window)
        else:
            o, lse = _ref_attention(q, k, v, causal, scale, cu_seqlens, seq_len, window)
        if AttnStash.mode == "record":
            AttnStash.items.append((o, lse))
        if _ap.tracking():  # per-tensor activation plan: qkv = RoPE(projection), recomputable; o / LSE are not
            if tagged is not None and tagged.fn is not None:
                _ap.tag(qkv, "qkv", fn=_qkv_recipe(tagged.fn, NH, D, n_q + n_kv, cos, sin, seq_len, pos_ids),
                        srcs=tagged.srcs)
            else:
                _ap.tag(qkv, "qkv")
            _ap.tag(o, "attn_out")
            _ap.tag(lse, "attn_lse")
        ctx.save_for_backward(qkv, o, lse, cos, sin, cu_seqlens, pos_ids)
        ctx.args = (n_q, n_kv, seq_len, causal, scale, window)
        return o.view(T, n_q * D)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, cos, sin, cu_seqlens, pos_ids = ctx.saved_tensors
        n_q, n_kv, seq_len, causal, scale, window = ctx.args
        T, NH, D = qkv.shape
        do = do.reshape(T, n_q, D).contiguous()
        q = qkv[:, :n_q]
        k = qkv[:, n_q:n_q + n_kv]
        v = qkv[:, n_q + n_kv:]
        dqkv = torch.empty_like(qkv)
        cu, B, sl, max_len = _cu_info(cu_seqlens, T, seq_len)
        if native_supported(qkv):
            _native_bwd(q, k, v, o, lse, do, dqkv[:, :n_q], dqkv[:, n_q:n_q + n_kv], dqkv[:, n_q + n_kv:], causal, scale,
                        cu, B, sl, max_len, window)
        else:
            dq, dk, dv = _ref_bwd(q, k, v, do, causal, scale, cu_seqlens, seq_len, window)
            dqkv[:, :n_q] = dq.to(qkv.dtype)
            dqkv[:, n_q:n_q + n_kv] = dk.to(qkv.dtype)
            dqkv[:, n_q + n_kv:] = dv.to(qkv.dtype)
        if cos is not None:
            rope_(dqkv, cos, sin, n_q + n_kv, seq_len=seq_len, pos_ids=pos_ids, sign=-1.0)
        return dqkv, None, None, None, None, None, None, None, None, None, None


def qkv_attention(qkv, n_q, n_kv, cos=None, sin=None, seq_len=None, causal=True, softmax_scale=None, cu_seqlens=None,
                  pos_ids=None, window=0):
    """qkv: [T, n_q + 2*n_kv, D] (fused projection output, CONSUMED: RoPE is applied in place).

    Returns the attention output flattened to [T, n_q * D] (ready for the O projection).
    """
    T, NH, D = qkv.shape
    assert NH == n_q + 2 * n_kv
    qkv = qkv if qkv.is_contiguous() else qkv.contiguous()
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    _count_attn_flops(T, n_q, D, int(seq_len or T), causal, cu_seqlens)
    return _QKVAttnFn.apply(qkv, n_q, n_kv, cos, sin, int(seq_len or T), bool(causal), float(scale), cu_seqlens,
                            pos_ids, int(window or 0))


# ---------------------------------------------------------------------------------------------
# Block primitives for chunked / blockwise attention (FPDT, ring-style merges). No autograd: the
# caller owns the global (o, lse) and calls the block backward once per (query-chunk, key-chunk) pair.
def _ref_block_bwd(q, k, v, o, lse, do, causal, scale, seq_len):
    """fp32 blockwise backward against an externally supplied (final) o / lse: P = exp(qk^T*scale - lse)."""
    T, Hq, D = q.shape
    Hkv = k.shape[1]
    G = Hq // Hkv
    B = T // seq_len
    L = seq_len

    def bh(t):  # [T, H, D] -> [B, H, L, D]
        return t.float().view(B, L, t.shape[1], D).permute(0, 2, 1, 3)

    qf, kf, vf, of, dof = bh(q), bh(k).repeat_interleave(G, 1), bh(v).repeat_interleave(G, 1), bh(o), bh(do)
    lsef = lse.float().view(Hq, B, L).permute(1, 0, 2)[..., None]  # [B, H, L, 1]
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        i = torch.arange(L, device=q.device)
        s = s.masked_fill(i[None, :] > i[:, None], float("-inf"))
    p = torch.exp(s - lsef)
    dv = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, kf)
    dk = torch.matmul(ds.transpose(-1, -2), qf)

    def tok(t, H):  # [B, H, L, D] -> [T, H, D]
        return t.permute(0, 2, 1, 3).reshape(T, H, D)

    dk = dk.view(B, Hkv, G, L, D).sum(2)
    dv = dv.view(B, Hkv, G, L, D).sum(2)
    return tok(dq, Hq), tok(dk, Hkv), tok(dv, Hkv)


def attn_block_fwd(q, k, v, causal, scale, seq_len):
    """One (query block, key block) FlashAttention forward on [T, H, D] tensors holding T/seq_len equal-length
    sequences; returns (o [T, Hq, D] in q.dtype, lse [Hq, T] fp32)."""
    T, Hq, D = q.shape
    if native_supported(q):
        o = torch.empty(T, Hq, D, device=q.device, dtype=q.dtype)
        lse = torch.empty(Hq, T, device=q.device, dtype=torch.float32)
        _native_fwd(q, k, v, o, lse, causal, scale, None, T // seq_len, seq_len, seq_len, 0)
        return o, lse
    return _ref_attention(q, k, v, causal, scale, None, seq_len, 0)


def attn_block_bwd(q, k, v, o, lse, do, causal, scale, seq_len):
    """Gradient contribution of one (query block, key block) pair given the FINAL merged o / lse of the query
    block (exact blockwise decomposition). Returns (dq, dk, dv); bf16 on the HIP path, fp32 on the reference."""
    T = q.shape[0]
    if native_supported(q):
        dq = torch.empty(q.shape, device=q.device, dtype=q.dtype)
        dk = torch.empty(k.shape, device=k.device, dtype=k.dtype)
        dv = torch.empty(v.shape, device=v.device, dtype=v.dtype)
        _native_bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale, None, T // seq_len, seq_len, seq_len, 0)
        return dq, dk, dv
    return _ref_block_bwd(q, k, v, o, lse, do, causal, scale, seq_len)


def padding_mask_lengths(mask, seq_len):
    """Valid lengths ``[B]`` if an additive attention mask ([B, 1, 1, S] or [B, S]; 0 = keep, large negative =
    drop) is a right-padding key mask, else None (the caller then needs a general masked attention)."""
    m = mask.reshape(mask.shape[0], -1) if mask.dim() == 4 and mask.shape[1] == 1 and mask.shape[2] == 1 else \
        (mask if mask.dim() == 2 else None)
    if m is None or m.shape[-1] != seq_len:
        return None
    keep = m > -1.0  # 0 keeps; masked positions hold -10000 / finfo.min
    lens = keep.sum(-1, dtype=torch.int32)
    prefix = torch.arange(seq_len, device=m.device)[None, :] < lens[:, None]
    if not bool(torch.equal(keep, prefix)) or bool((m[keep] != 0).any()):
        return None
    return lens


def merge_attn_out(o, lse, o_blk, lse_blk):
    """Online-softmax merge of two partial attention results (fp32 o [T, H, D], lse [H, T])."""
    if o is None:
        return o_blk.float(), lse_blk.clone()
    new = torch.logaddexp(lse, lse_blk)
    a = torch.exp(lse - new).t()[..., None]
    b = torch.exp(lse_blk - new).t()[..., None]
    return o * a + o_blk.float() * b, new
