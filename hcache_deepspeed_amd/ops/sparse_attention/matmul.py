"""Block-sparse matmul and softmax over a layout's compressed block format.

Reference parity: ops/sparse_attention/matmul.py (``MatMul(layout, block, mode, trans_a, trans_b)`` with modes
``sdd`` (dense x dense -> sparse), ``dsd`` (sparse x dense -> dense), ``dds`` (dense x sparse -> dense); Triton
kernels there) and ops/sparse_attention/softmax.py (``Softmax(layout, block)``: row softmax over the non-zero
blocks with scale, relative-position embedding, key-padding and attention masks).

Compressed format: ``[B, nnz, block, block]`` where block ``e`` is layout entry ``layout.nonzero()[e] = (h, r, c)``
(head-major, then row, then column -- the reference's ordering). Here the products are batched GEMMs over the
gathered blocks (hipBLASLt through torch.matmul) and the row reductions are scatter-reduces; every op is
differentiable through autograd. The fused flash-style HIP kernel (sparse_attn.hip, used by
:class:`SparseSelfAttention` for 64-multiple blocks) never materialises this format at all.
"""
import torch


class _Layout:

    def __init__(self, layout, block):
        layout = layout.to(torch.int64)
        self.layout = layout
        self.block = block
        self.H, self.nb_r, self.nb_c = layout.shape
        nz = layout.nonzero()
        self.h, self.r, self.c = nz[:, 0], nz[:, 1], nz[:, 2]
        self.nnz = nz.shape[0]
        self._dev = {}

    def idx(self, device):
        if device not in self._dev:
            self._dev[device] = (self.h.to(device), self.r.to(device), self.c.to(device))
        return self._dev[device]


def _blocks_rows(x, H, nb, block):
    """[B, H, nb*block, K] -> [B, H, nb, block, K]"""
    B, _, _, K = x.shape
    return x.reshape(B, H, nb, block, K)


class MatMul:
    """Block-sparse matrix multiplication; ``mode`` in {'sdd', 'dsd', 'dds'} (see module docstring)."""

    def __init__(self, layout, block, mode, trans_a=False, trans_b=False, bench=False):
        if mode not in ("sdd", "dsd", "dds"):
            raise NotImplementedError("Supported modes are: sdd, dsd, dds")
        self.lay = _Layout(layout, block)
        self.block, self.mode = block, mode
        self.trans_a, self.trans_b = trans_a, trans_b

    def __call__(self, a, b):
        L, blk = self.lay, self.block
        if self.mode == "sdd":
            a = a.transpose(-1, -2) if self.trans_a else a
            b = b.transpose(-1, -2) if self.trans_b else b
            h, r, c = L.idx(a.device)
            ab = _blocks_rows(a, a.shape[1], L.nb_r, blk)[:, h % a.shape[1], r]  # [B, nnz, blk, K]
            bt = _blocks_rows(b.transpose(-1, -2), b.shape[1], L.nb_c, blk)[:, h % b.shape[1], c]  # [B, nnz, blk, K]
            return torch.matmul(ab, bt.transpose(-1, -2))
        if self.mode == "dsd":  # a sparse [B, nnz, blk, blk] (M x K blocks), b dense [B, H, K, N]
            b = b.transpose(-1, -2) if self.trans_b else b
            h, r, c = L.idx(b.device)
            x = a.transpose(-1, -2) if self.trans_a else a
            rows, cols = (c, r) if self.trans_a else (r, c)
            nb_out = L.nb_c if self.trans_a else L.nb_r
            B, H, _, N = b.shape
            bb = _blocks_rows(b, H, b.shape[2] // blk, blk)[:, h % H, cols]  # [B, nnz, blk, N]
            prod = torch.matmul(x, bb)  # [B, nnz, blk, N]
            out = torch.zeros(B, H * nb_out, blk, N, dtype=prod.dtype, device=prod.device)
            out = out.index_add(1, h * nb_out + rows, prod)
            return out.view(B, H, nb_out * blk, N)
        # dds: a dense [B, H, M, K], b sparse [B, nnz, blk, blk] (K x N blocks)
        a = a.transpose(-1, -2) if self.trans_a else a
        h, r, c = L.idx(a.device)
        x = b.transpose(-1, -2) if self.trans_b else b
        krow, ncol = (c, r) if self.trans_b else (r, c)
        nb_out = L.nb_r if self.trans_b else L.nb_c
        B, H, M, K = a.shape
        ab = a.reshape(B, H, M, K // blk, blk).permute(0, 1, 3, 2, 4)[:, h % H, krow]  # [B, nnz, M, blk]
        prod = torch.matmul(ab, x)  # [B, nnz, M, blk]
        out = torch.zeros(B, H * nb_out, M, blk, dtype=prod.dtype, device=prod.device)
        out = out.index_add(1, h * nb_out + ncol, prod)
        return out.view(B, H, nb_out, M, blk).permute(0, 1, 3, 2, 4).reshape(B, H, M, nb_out * blk)


class Softmax:
    """Row softmax over the non-zero blocks of each layout row (compressed format in/out)."""

    def __init__(self, layout, block, bench=False):
        self.lay = _Layout(layout, block)
        self.block = block

    def __call__(self, x, scale=1.0, rpe=None, key_padding_mask=None, attn_mask=None, key_padding_mask_mode="add",
                 attn_mask_mode="add"):
        L, blk = self.lay, self.block
        h, r, c = L.idx(x.device)
        B = x.shape[0]
        s = x.float() * scale
        qpos = (r[:, None] * blk + torch.arange(blk, device=x.device)[None, :])  # [nnz, blk]
        kpos = (c[:, None] * blk + torch.arange(blk, device=x.device)[None, :])
        if rpe is not None:  # [H, S, S] (or broadcastable) dense relative-position bias
            rp = rpe if rpe.dim() == 3 else rpe.reshape(-1, rpe.shape[-2], rpe.shape[-1])
            s = s + rp[(h % rp.shape[0])[:, None, None], qpos[:, :, None], kpos[:, None, :]].float()
        if key_padding_mask is not None:  # [B, S]
            km = key_padding_mask[:, kpos].float()[:, :, None, :]  # [B, nnz, 1, blk]
            s = s + km if key_padding_mask_mode == "add" else s.masked_fill(km == 0, float("-inf"))
        if attn_mask is not None:  # [S, S]
            am = attn_mask[qpos[:, :, None], kpos[:, None, :]].float()[None]
            s = s + am if attn_mask_mode == "add" else s.masked_fill(am == 0, float("-inf"))
        row = (h * L.nb_r + r)  # [nnz]
        nrows = L.H * L.nb_r
        # per-(batch, row, query) max over all blocks of the row
        mx = torch.full((B, nrows, blk), float("-inf"), device=x.device)
        mx = mx.scatter_reduce(1, row[None, :, None].expand(B, -1, blk), s.amax(-1), "amax", include_self=True)
        mx = torch.where(torch.isinf(mx), torch.zeros_like(mx), mx)
        e = torch.exp(s - mx[:, row][..., None])
        den = torch.zeros(B, nrows, blk, device=x.device).index_add(1, row, e.sum(-1))
        out = e / den[:, row][..., None].clamp_min(1e-30)
        return out.to(x.dtype)
