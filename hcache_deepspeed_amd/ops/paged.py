"""Paged-KV serving ops: fused RoPE + KV scatter, ragged paged attention (HIP, csrc/kernels/paged_attn.hip).

Reference parity: inference/v2/kernels/ragged_ops/linear_blocked_kv_rotary (``LinearBlockedKVCopy``,
``BlockedRotaryEmbeddings``) and ragged_ops/blocked_flash (``BlockedFlashAttn``) + atom_builder.
CPU tensors run torch references (used by the CPU test-suite and as the GPU numerics oracle).
"""
import torch

from . import native

ROWS_PER_ATOM = 128


def kernel_head_dim_ok(D):
    """The HIP serving kernels are instantiated for the same head dims as the training FlashAttention."""
    from .attention import head_dim_supported
    return head_dim_supported(D)


def kv_rope_scatter(qkv, cache, tok_seq, tok_pos, block_tables, cos, sin, n_q, n_kv, rotate_q=True, do_rope=True,
                    rotary_dim=0):
    """qkv: [T, n_q + 2 n_kv, D]; cache: [num_blocks, block_size, 2, n_kv, D] (one layer).

    RoPE at absolute positions ``tok_pos`` on q (in place, if ``rotate_q``) and k (the first ``rotary_dim``
    dims only when 0 < rotary_dim < D: partial rotary of Phi / GPT-NeoX style models); k and v are written
    to ``cache[block_tables[tok_seq[t], pos // bs], pos % bs]``.
    """
    T, NH, D = qkv.shape
    bs = cache.shape[1]
    partial = do_rope and 0 < rotary_dim < D
    if native.use_native(qkv):
        rd = rotary_dim if partial else D
        if D % 4 or rd % 8:
            raise NotImplementedError(f"kv_rope_scatter: head_dim {D} / rotary_dim {rd} not supported on the GPU")
        native.check(
            native.kernels().hds_kv_rope_scatter(native.dt(qkv), qkv.data_ptr(), qkv.stride(0), cache.data_ptr(),
                                                 tok_seq.data_ptr(), tok_pos.data_ptr(), block_tables.data_ptr(),
                                                 block_tables.shape[1], cos.data_ptr() if do_rope else None,
                                                 sin.data_ptr() if do_rope else None, T, n_q, n_kv, D, rd, bs,
                                                 int(rotate_q), int(do_rope), native.stream()), "kv_rope_scatter")
        return
    pos = tok_pos.long()
    rd = rotary_dim if partial else D
    half = rd // 2

    def rot(x):
        if not do_rope:
            return x
        c = cos[pos][:, None, :half]
        s = sin[pos][:, None, :half]
        xf = x[..., :rd].float()
        a, b = xf[..., :half], xf[..., half:]
        r = torch.cat([a * c - b * s, b * c + a * s], -1).to(x.dtype)
        return torch.cat([r, x[..., rd:]], -1) if rd < D else r

    if rotate_q:
        qkv[:, :n_q] = rot(qkv[:, :n_q])
    k = rot(qkv[:, n_q:n_q + n_kv])
    v = qkv[:, n_q + n_kv:]
    blk = block_tables[tok_seq.long(), pos // bs].long()
    slot = pos % bs
    cache[blk, slot, 0] = k
    cache[blk, slot, 1] = v


def build_atoms(seq_meta_host, n_q, n_kv):
    """seq_meta_host: list of (q_start, n_new, seen). Returns int32 [n_atoms, 3] = (seq, kv_head, row_start)."""
    G = n_q // n_kv
    atoms = []
    for s, (_, n_new, _) in enumerate(seq_meta_host):
        rows = n_new * G
        for hk in range(n_kv):
            for r0 in range(0, rows, ROWS_PER_ATOM):
                atoms.append((s, hk, r0))
    return torch.tensor(atoms if atoms else [(0, 0, 0)], dtype=torch.int32), len(atoms)


_COUNTERS = {}
_MERGE_IN_KERNEL = __import__("os").environ.get("HDS_DECODE_MERGE_IN_KERNEL", "0") == "1"


def _merge_counters(device, n):
    """Per-device ints the split-K decode kernel counts finished splits in (the last workgroup of a (sequence, kv
    head) merges the splits and zeroes its counter again): allocated once, zeroed, with room for 64K (sequence, kv
    head) pairs, so a HIP-graph decode captures a stable address. ``HDS_DECODE_MERGE_IN_KERNEL=1`` turns it on;
    by default the separate combine launch merges: the device-scope release each split workgroup needs (its L2
    written back for the other XCDs) cost more than the saved launch -- v2 decode B = 1 200 vs 247 tok/s, B = 8
    1,096 vs 1,490 (profiles/r6/decode_merge/)."""
    if not _MERGE_IN_KERNEL or n > 65536:
        return None
    buf = _COUNTERS.get(device)
    if buf is None:
        buf = _COUNTERS[device] = torch.zeros(65536, dtype=torch.int32, device=device)
    return buf.data_ptr()


def paged_attention(q, cache, atoms, n_atoms, seq_meta, block_tables, n_q, n_kv, scale, window=0,
                    seq_meta_host=None, block_tables_host=None, decode=False):
    """q: [T, n_q, D] (token-strided view ok). Returns o [T, n_q, D]. ``decode``: every sequence of the batch has
    exactly one new token (T == n_seqs) -- the split-K paged decode kernel runs instead of the atom kernel; its key
    splits are sized from the cache capacity (block table width x block size), so one launch shape serves every
    step of a HIP-graph decode."""
    T, _, D = q.shape
    o = torch.empty(T, n_q, D, device=q.device, dtype=q.dtype)
    if native.use_native(q):
        if not kernel_head_dim_ok(D) or q.dtype != torch.bfloat16:
            raise NotImplementedError(f"paged_attention: head_dim {D} / {q.dtype} has no HIP kernel")
        lib = native.kernels()
        if decode and lib.hds_paged_decode_supported(D, n_q // n_kv):
            n_seqs = T
            splits = lib.hds_paged_decode_splits(n_seqs, n_kv, block_tables.shape[1] * cache.shape[1])
            part_o = part_ml = None
            if splits > 1:
                part_o = torch.empty(n_seqs * n_q * splits * D, device=q.device, dtype=torch.float32)
                part_ml = torch.empty(n_seqs * n_q * splits * 2, device=q.device, dtype=torch.float32)
            native.check(
                lib.hds_paged_decode(q.data_ptr(), q.stride(0), cache.data_ptr(), o.data_ptr(), native.ptr(part_o),
                                     native.ptr(part_ml), seq_meta.data_ptr(), block_tables.data_ptr(),
                                     block_tables.shape[1], cache.shape[1], n_seqs, n_q, n_kv, D, splits, float(scale),
                                     int(window), _merge_counters(q.device, n_seqs * n_kv) if splits > 1 else None,
                                     native.stream()), "paged_decode")
            return o
        native.check(
            lib.hds_paged_attn(q.data_ptr(), q.stride(0), cache.data_ptr(), o.data_ptr(), atoms.data_ptr(), n_atoms,
                               seq_meta.data_ptr(), block_tables.data_ptr(), block_tables.shape[1], cache.shape[1],
                               n_q, n_kv, D, float(scale), int(window), native.stream()), "paged_attn")
        return o
    meta = seq_meta_host if seq_meta_host is not None else seq_meta.tolist()
    tables = block_tables_host if block_tables_host is not None else block_tables
    bs = cache.shape[1]
    G = n_q // n_kv
    for s, (q0, n_new, seen) in enumerate(meta):
        if n_new == 0:
            continue
        ctx = seen + n_new
        pos = torch.arange(ctx, device=q.device)
        blk = torch.as_tensor(tables[s], device=q.device)[pos // bs].long()
        kk = cache[blk, pos % bs, 0].float()  # [ctx, n_kv, D]
        vv = cache[blk, pos % bs, 1].float()
        qq = q[q0:q0 + n_new].float()  # [n_new, n_q, D]
        kk = kk.repeat_interleave(G, 1)
        vv = vv.repeat_interleave(G, 1)
        sc = torch.einsum("thd,chd->htc", qq, kk) * scale
        qpos = seen + torch.arange(n_new, device=q.device)
        mask = pos[None, :] > qpos[:, None]
        if window:
            mask |= pos[None, :] <= qpos[:, None] - window
        sc = sc.masked_fill(mask[None], float("-inf"))
        o[q0:q0 + n_new] = torch.einsum("htc,chd->thd", torch.softmax(sc, -1), vv).to(o.dtype)
    return o
