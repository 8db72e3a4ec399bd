"""Block-sparse self-attention module.

Reference parity: ops/sparse_attention/sparse_self_attention.py (``SparseSelfAttention(sparsity_config,
key_padding_mask_mode='add', attn_mask_mode='mul', max_seq_length=2048)``; forward(query, key, value, rpe,
key_padding_mask, attn_mask) on [B, H, S, D]; layouts cached per sequence length; sdd -> softmax -> dsd).

Two execution paths:

* **HIP fused path** (``block_sparse_attention``): bf16 on GPU, head_dim 128, layout block a multiple of 64 and no
  rpe / masks -> csrc/kernels/sparse_attn.hip, a flash-style kernel that walks only the non-zero 64x64 blocks of
  each query row (fwd, dQ) or key column (dK/dV). Memory O(S*D), no score matrix.
* **compressed-format path** (any block size, rpe / key-padding / attention masks): MatMul('sdd') -> Softmax ->
  MatMul('dsd') of matmul.py, exactly the reference's decomposition.
"""
import math

import torch
import torch.nn as nn

from .. import native
from .matmul import MatMul, Softmax
from .sparsity_config import SparsityConfig

_NATIVE_BLOCK = 64


class _CSR:
    """64-granular CSR + CSC index arrays of a [Hl, nb, nb] layout, cached per device."""

    def __init__(self, layout):
        lay = layout.to(torch.int64)
        self.layout_heads, self.nb = lay.shape[0], lay.shape[1]
        rows, cols = [], []
        rp, ci, cp, ri = [], [], [], []
        for h in range(self.layout_heads):
            m = lay[h] != 0
            rp.append(torch.cat([torch.zeros(1, dtype=torch.int64), m.sum(1).cumsum(0)]))
            ci.append(m.nonzero()[:, 1])
            mt = m.t()
            cp.append(torch.cat([torch.zeros(1, dtype=torch.int64), mt.sum(1).cumsum(0)]))
            ri.append(mt.nonzero()[:, 1])
        off_r = torch.tensor([0] + [len(x) for x in ci]).cumsum(0)
        off_c = torch.tensor([0] + [len(x) for x in ri]).cumsum(0)
        self.row_ptr = torch.cat([rp[h] + off_r[h] for h in range(self.layout_heads)]).to(torch.int32)
        self.col_ptr = torch.cat([cp[h] + off_c[h] for h in range(self.layout_heads)]).to(torch.int32)
        self.col_idx = torch.cat(ci).to(torch.int32) if ci else torch.zeros(0, dtype=torch.int32)
        self.row_idx = torch.cat(ri).to(torch.int32) if ri else torch.zeros(0, dtype=torch.int32)
        self._dev = {}

    def on(self, device):
        if device not in self._dev:
            t = [x.to(device) if x.numel() else torch.zeros(1, dtype=torch.int32, device=device)
                 for x in (self.row_ptr, self.col_idx, self.col_ptr, self.row_idx)]
            self._dev[device] = t
        return self._dev[device]


def _strides8(*ts):
    vals = [0 if t is None else t.stride(0) for t in ts]
    vals += [0] * (8 - len(vals))
    return torch.tensor(vals, dtype=torch.int64)


class _BSAttnFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, k, v, csr, B, S, causal, scale):
        # q/k/v: [B*S, H, 128] token-major
        T, Hq, D = q.shape
        rp, ci, cp, ri = csr.on(q.device)
        o = torch.empty_like(q)
        lse = torch.empty(Hq, T, dtype=torch.float32, device=q.device)
        strides = _strides8(q, k, v, o)  # host array read by the launcher: keep it alive across the call
        native.check(native.kernels().hds_bsattn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                                     lse.data_ptr(), strides.data_ptr(), rp.data_ptr(),
                                                     ci.data_ptr(), csr.layout_heads, csr.nb, B, S, Hq, k.shape[1], D,
                                                     float(scale), int(causal), native.stream()), "bsattn_fwd")
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.args = (csr, B, S, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        csr, B, S, causal, scale = ctx.args
        do = do.contiguous()
        T, Hq, D = q.shape
        rp, ci, cp, ri = csr.on(q.device)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty(Hq, T, dtype=torch.float32, device=q.device)
        strides = _strides8(q, k, v, o, do, dq, dk, dv)
        native.check(
            native.kernels().hds_bsattn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                                            do.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                                            delta.data_ptr(), strides.data_ptr(),
                                            rp.data_ptr(), ci.data_ptr(), cp.data_ptr(), ri.data_ptr(),
                                            csr.layout_heads, csr.nb, B, S, Hq, k.shape[1], D, float(scale),
                                            int(causal), native.stream()), "bsattn_bwd")
        return dq, dk, dv, None, None, None, None, None


def native_layout(layout, block):
    """Re-express a ``block``-granular layout at the kernel's 64 granularity (block must be a multiple of 64)."""
    assert block % _NATIVE_BLOCK == 0
    f = block // _NATIVE_BLOCK
    return layout.repeat_interleave(f, 1).repeat_interleave(f, 2) if f > 1 else layout


def block_sparse_attention(q, k, v, layout, block, causal=False, softmax_scale=None, csr=None):
    """Fused block-sparse attention. q: [B, Hq, S, D]; k/v: [B, Hkv, S, D]; layout [Hl, S/block, S/block] with
    Hl in {1, Hq}. HIP kernel when eligible, compressed-format torch path otherwise. Returns [B, Hq, S, D]."""
    B, Hq, S, D = q.shape
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    if q.is_cuda and q.dtype == torch.bfloat16 and D == 128 and block % _NATIVE_BLOCK == 0:
        if csr is None:
            csr = _CSR(native_layout(layout, block))
        assert S == csr.nb * _NATIVE_BLOCK and csr.layout_heads in (1, Hq) and Hq % k.shape[1] == 0, \
            f"block-sparse kernel: S={S} vs {csr.nb} blocks of 64, layout heads {csr.layout_heads} vs Hq={Hq}"
        qt, kt, vt = (x.transpose(1, 2).reshape(B * S, x.shape[1], D) for x in (q, k, v))
        o = _BSAttnFn.apply(qt.contiguous(), kt.contiguous(), vt.contiguous(), csr, B, S, bool(causal), scale)
        return o.view(B, S, Hq, D).transpose(1, 2)
    lay = layout if layout.shape[0] == Hq else layout.expand(Hq, -1, -1)
    if causal:
        lay = torch.tril(lay)
    G = Hq // k.shape[1]
    if G > 1:
        k, v = k.repeat_interleave(G, 1), v.repeat_interleave(G, 1)
    sdd, dsd, sm = MatMul(lay, block, "sdd", trans_b=True), MatMul(lay, block, "dsd"), Softmax(lay, block)
    s = sdd(q, k)
    am = None
    if causal:
        am = torch.tril(torch.ones(S, S, device=q.device))
    p = sm(s, scale=scale, attn_mask=am, attn_mask_mode="mul")
    return dsd(p, v)


class SparseSelfAttention(nn.Module):
    """Efficient block-sparse self-attention (reference SparseSelfAttention)."""

    def __init__(self, sparsity_config=None, key_padding_mask_mode="add", attn_mask_mode="mul",
                 max_seq_length=2048):
        super().__init__()
        self.sparsity_config = sparsity_config if sparsity_config is not None else SparsityConfig(num_heads=4)
        self.key_padding_mask_mode = key_padding_mask_mode
        self.attn_mask_mode = attn_mask_mode
        self.max_seq_length = max_seq_length
        self._layouts = {}
        self._ops = {}
        self._csr = {}

    def get_layout(self, L):
        if L % self.sparsity_config.block != 0:
            raise ValueError(f"Sequence Length, {L}, needs to be dividable by Block size "
                             f"{self.sparsity_config.block}!")
        if L not in self._layouts:
            self._layouts[L] = self.sparsity_config.make_layout(L)
        return self._layouts[L]

    def get_ops(self, H, L):
        if L not in self._ops:
            lay, blk = self.get_layout(L), self.sparsity_config.block
            self._ops[L] = (MatMul(lay, blk, "sdd", trans_a=False, trans_b=True), MatMul(lay, blk, "dsd"),
                            Softmax(lay, blk))
        return self._ops[L]

    def transpose_key_for_scores(self, x, L):
        bsz, num_heads, seq_len, head_dim = x.size()
        if seq_len != L:
            return x.permute(0, 1, 3, 2)
        return x

    def transpose_mask_for_sparse(self, qtype, x, is_key_padding_mask=False):
        x = x.type(qtype)
        if is_key_padding_mask:
            xdim = x.dim()
            for d in range(xdim - 1, 0, -1):
                x = x.squeeze(dim=d)
            return x
        return x.squeeze()

    def forward(self, query, key, value, rpe=None, key_padding_mask=None, attn_mask=None):
        """query/key/value: [B, H, S, D] -> [B, H, S, D]."""
        assert query.dtype in (torch.float16, torch.bfloat16, torch.float32)
        bsz, num_heads, tgt_len, head_dim = query.size()
        key = self.transpose_key_for_scores(key, tgt_len)
        if query.shape != key.shape or key.shape != value.shape:
            raise NotImplementedError("only self-attention is supported for now")
        blk = self.sparsity_config.block
        scaling = float(head_dim)**-0.5
        if (query.is_cuda and query.dtype == torch.bfloat16 and head_dim == 128 and blk % _NATIVE_BLOCK == 0
                and rpe is None and key_padding_mask is None and attn_mask is None):
            if tgt_len not in self._csr:
                self._csr[tgt_len] = _CSR(native_layout(self.get_layout(tgt_len), blk))
            return block_sparse_attention(query, key, value, self.get_layout(tgt_len), blk, causal=False,
                                          softmax_scale=scaling, csr=self._csr[tgt_len])
        if key_padding_mask is not None:
            key_padding_mask = self.transpose_mask_for_sparse(query.dtype, key_padding_mask,
                                                              is_key_padding_mask=True)
        if attn_mask is not None:
            attn_mask = self.transpose_mask_for_sparse(query.dtype, attn_mask)
        sdd, dsd, sm = self.get_ops(num_heads, tgt_len)
        s = sdd(query, key)
        p = sm(s, scale=scaling, rpe=rpe, key_padding_mask=key_padding_mask, attn_mask=attn_mask,
               key_padding_mask_mode=self.key_padding_mask_mode, attn_mask_mode=self.attn_mask_mode)
        return dsd(p, value)
